"""Per-kernel averages of rocprofv3 --pmc counters (SQ issue/wait breakdown of the decode GEMVs).
SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles (MI355X_MICROARCH.md, PMC table);
WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~= WAVE_CYCLES.
usage: python scripts/pmc_sq.py <counter_collection.csv> [kernel-substring ...]"""
import csv
import sys
from collections import defaultdict


def main():
    path, pats = sys.argv[1], sys.argv[2:] or ["gemv_kernel", "attn_fused"]
    acc = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(path)):
        k = r.get("Kernel_Name", "")
        if any(p in k for p in pats):
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in sorted(acc.items()):
        name = k.split("(")[0].replace("void ", "").replace("mi::(anonymous namespace)::", "")
        avg = {c: sum(v) / len(v) for c, v in d.items()}
        n = max(len(v) for v in d.values())
        line = " ".join(f"{c}={avg[c]:.4g}" for c in sorted(avg))
        wc = avg.get("SQ_WAVE_CYCLES")
        if wc:
            parts = [f"{c[3:]} {avg[c] / wc:.1%}" for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                                                          "SQ_ACTIVE_INST_VALU") if c in avg]
            line += " | " + ", ".join(parts)
        print(f"{name} x{n}: {line}")


if __name__ == "__main__":
    main()
