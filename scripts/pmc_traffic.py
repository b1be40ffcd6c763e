"""Per-launch HBM read traffic of the bench's roofline kernel from a rocprofv3 --pmc FETCH_SIZE
pass (MI355X_MICROARCH.md, HBM section: FETCH_SIZE counts 64 B per 128-B request of a wide
coalesced streaming read on gfx950, i.e. half the bytes -> doubled here; the unit is KB).
usage: python scripts/pmc_traffic.py <counter_collection.csv> <kernel-substring> <out.json> [bench-config]"""
import csv
import json
import sys


def main():
    path, pat, out = sys.argv[1], sys.argv[2], sys.argv[3]
    vals = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if pat in r.get("Kernel_Name", "") and r.get("Counter_Name") == "FETCH_SIZE":
                vals.append(float(r["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no FETCH_SIZE rows for kernels matching {pat!r}")
    avg_kb = sum(vals) / len(vals)
    res = {"kernel_match": pat, "launches": len(vals), "fetch_size_kb_avg": avg_kb,
           "traffic_bytes_per_launch": avg_kb * 1024 * 2,
           "correction": "x2: gfx950 FETCH_SIZE reports half the bytes of 16-B/lane streaming reads",
           "config": sys.argv[4] if len(sys.argv) > 4 else "llama2-7b-q4_k_m"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
