"""Per-kernel time of the bench's short verification legs in an eager kernel trace
(rocprofv3 --kernel-trace csv): the last two runs of consecutive short-batch kernels."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
keys = ("mmqs_t", "qkv_finish", "part_sum", "quant_act", "attn_mfma", "attn_fused", "embed_multi", "rope_table")
segs, cur = [], []
for r in rows:
    if any(k in r["Kernel_Name"] for k in keys):
        cur.append(r)
    else:
        if len(cur) > 50 and any("mmqs_t" in x["Kernel_Name"] for x in cur):
            segs.append(cur)
        cur = []
if len(cur) > 50:
    segs.append(cur)
for s in segs[-2:]:
    agg, cnt = collections.defaultdict(float), collections.defaultdict(int)
    for r in s:
        n = r["Kernel_Name"].replace("mi::mmq::", "").replace("mi::", "").split("(")[0][:45]
        agg[n] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
        cnt[n] += 1
    print("kernel sum us", round(sum(agg.values()), 1))
    for n in sorted(agg, key=lambda k: -agg[k]):
        print(f"  {n:45s} {cnt[n]:4d} x {agg[n] / cnt[n]:7.2f} = {agg[n]:8.1f}")
