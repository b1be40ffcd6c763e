"""Regenerate tests/golden/oracle_golden.npz from the numpy oracle.

These are regression fixtures of OUR restatement (the reference holds no
golden vectors for the quant formats -- SURVEY.md §8c5, "parity unpinned");
the only reference-held known answer is the LogitComparer KAT, asserted
directly in tests/test_oracle.py.
Run: python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import ggml_ref as R  # noqa: E402
from util import QTYPES, rand_matrix, rand_x, oracle_from_gguf  # noqa: E402
from blama_amd import synthetic  # noqa: E402

out = {}
for t in QTYPES:
    K = 512
    w = rand_matrix(t, 4, K, seed=100 + t)
    x = rand_x(K, seed=200 + t)
    out[f"w_{t}"] = w
    out[f"x_{t}"] = x
    out[f"deq_{t}"] = R.dequantize(w, t)
    out[f"y_{t}"] = R.mul_mat_vec(w, t, K, x)
xq = rand_x(768, seed=5, scale=2.0)
qk = R.quantize_q8_K(xq)
out["xq"] = xq
out["q8k_qs"] = qk.qs.reshape(-1).astype(np.int8)
out["q8k_d"] = qk.d
prompt = np.array([1, 5, 77, 300, 12], np.int32)
o = oracle_from_gguf(synthetic.build_gguf(synthetic.CONFIGS["tiny-q4_k_m"], seed=11), n_ctx=16)
out["prompt"] = prompt
out["logits"] = o.decode(list(prompt))
np.savez_compressed(os.path.join(HERE, "oracle_golden.npz"), **out)
print("wrote", os.path.join(HERE, "oracle_golden.npz"))
