"""GEMV micro-benchmark over the decode shapes, through the
C ABI's mi_op_gemv_bench (median device time of single launches, matrix copies
rotated so that every launch streams from HBM, not the Infinity Cache).

Usage: python scripts/gemv_sweep.py [cfg ...]   (cfg = MI_GEMV_CFG values; each
in its own process since the engine reads the variable once)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = [  # (type, rows, K)
    (12, 4096, 4096), (12, 12288, 4096), (12, 11008, 4096), (12, 22016, 4096), (12, 4096, 11008),
    (14, 4096, 4096), (14, 4096, 11008), (14, 32000, 4096), (14, 1024, 4096), (14, 14336, 4096),
    (14, 128256, 4096), (13, 14336, 4096), (13, 4096, 14336), (8, 2048, 2048), (8, 32000, 2048),
]
BB = {12: (256, 144), 13: (256, 176), 14: (256, 210), 8: (32, 34)}


def run_one():
    import numpy as np
    from blama_amd import engine, synthetic
    out = []
    for t, rows, K in SHAPES:
        be, bb = BB[t]
        raw = np.zeros(rows * (K // be) * bb, np.uint8)
        synthetic.fill_quant(raw, t, np.random.default_rng(0))
        us = engine.op_gemv_bench(t, raw, rows, K, iters=50)
        nbytes = rows * (K // be) * bb + K * 4 + rows * 4
        out.append({"type": t, "rows": rows, "K": K, "us": round(us, 2), "GBps": round(nbytes / us / 1e3, 1)})
    return out


def main():
    if os.environ.get("GEMV_SWEEP_CHILD"):
        print(json.dumps(run_one()))
        return
    cfgs = sys.argv[1:] or ["-1"]
    res = {}
    for c in cfgs:
        env = dict(os.environ, GEMV_SWEEP_CHILD="1")
        if c != "-1":
            env["MI_GEMV_CFG"] = c
        p = subprocess.run([sys.executable, __file__], env=env, capture_output=True, text=True, timeout=240)
        if p.returncode != 0:
            print(f"cfg {c} failed rc={p.returncode}: {p.stderr[-2000:]}")
            sys.exit(p.returncode)
        res[c] = json.loads(p.stdout.strip().splitlines()[-1])
    hdr = "type  rows    K     " + "  ".join(f"cfg{c:>3}: us / GB/s" for c in cfgs)
    print(hdr)
    for i, (t, rows, K) in enumerate(SHAPES):
        cols = "  ".join(f"{res[c][i]['us']:8.2f} / {res[c][i]['GBps']:6.0f}" for c in cfgs)
        print(f"{t:4d} {rows:6d} {K:6d}  {cols}")


if __name__ == "__main__":
    main()
