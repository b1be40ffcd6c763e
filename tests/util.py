"""Shared test helpers: seeded random quant matrices and synthetic models."""
import numpy as np

import ggml_ref as R
from blama_amd import gguf, synthetic

QTYPES = [R.Q4_K, R.Q5_K, R.Q6_K, R.Q8_0]


def rand_matrix(t: int, rows: int, K: int, seed: int = 0, std: float = 0.03) -> np.ndarray:
    buf = np.empty(R.row_bytes(t, K) * rows, np.uint8)
    synthetic.fill_quant(buf, t, np.random.default_rng(seed), std=std)
    return buf


def rand_x(K: int, seed: int = 1, scale: float = 1.0) -> np.ndarray:
    return (np.random.default_rng(seed).standard_normal(K) * scale).astype(np.float32)


def oracle_from_gguf(buf, n_ctx: int = 0) -> R.LlamaOracle:
    rd = gguf.GGUFReader(buf)
    kv = rd.kv
    a = kv["general.architecture"]
    n_embd = int(kv[f"{a}.embedding_length"])
    n_head = int(kv[f"{a}.attention.head_count"])
    te = rd.tensors["token_embd.weight"]
    hp = R.HParams(
        n_vocab=int(te.shape[1]), n_embd=n_embd, n_layer=int(kv[f"{a}.block_count"]),
        n_head=n_head, n_head_kv=int(kv.get(f"{a}.attention.head_count_kv", n_head)),
        n_ff=int(kv[f"{a}.feed_forward_length"]), n_ctx_train=int(kv[f"{a}.context_length"]),
        eps=float(kv.get(f"{a}.attention.layer_norm_rms_epsilon", kv.get(f"{a}.attention.layer_norm_epsilon", 1e-5))),
        rope_base=float(kv.get(f"{a}.rope.freq_base", 10000.0)),
        n_rot=int(kv.get(f"{a}.rope.dimension_count", n_embd // n_head)),
        n_expert=int(kv.get(f"{a}.expert_count", 0)), n_expert_used=int(kv.get(f"{a}.expert_used_count", 0)),
        arch=a)
    tens = {k: R.Tensor(v.type, v.shape, v.data) for k, v in rd.tensors.items()}
    return R.LlamaOracle(hp, tens, n_ctx=n_ctx)


def oracle_ulp_floor(buf, n_ctx, prompt, tokens, runs=4, seed=100):
    """The live rounding floor of the CPU algorithm at each output of a decode run.

    The oracle is re-run `runs` times with every GEMV output moved by -1, 0 or +1 ulp at random:
    an fp32 summation order exactly as valid as ggml's (its AVX2 and generic paths differ in
    it).  Returns base outputs and, per output (the prompt's last token, then each of `tokens`),
    the largest max|perturbed - base| over the runs.  A step where the HIP engine differs from the
    oracle by more than the element-wise tolerance is still at parity when the oracle itself moves
    that far under a 1-ulp change: a Q8_K / Q8_0 activation quantum or an f16 rounding (GELU
    table index, attention weight) sat on its boundary and flipped (measured for tiny-gpt2 step 7:
    1.2e-2 x rms in 3 of 4 perturbed runs, every other step <= 3e-6).  The perturbed runs also
    accumulate the attention dots (KQ, KQV) in f32 as ggml's AVX2 ggml_vec_dot_f16 does, where
    the base oracle sums in double, and move every score and head output by -1/0/+1 ulp: the synthetic GPT-2 models have large, flat attention scores
    past ~500 cells, where that alone moves the oracle's logits by 7.7e-3 x rms
    (tiny-gpt2-q8_0, 520 cells).  F32 weights (the MoE router, summed in double by the base
    oracle) are summed in f32 in the perturbed runs: a router near-tie there picks another
    expert (tiny-moe row 35: 5.4e-3 x rms, GPU batch and per-token paths alike)."""
    orig = R.mul_mat_vec
    orig_attn = R.attention_head

    def ulp(y, rng):
        y = np.ascontiguousarray(y, np.float32)
        return (y.view(np.int32) + rng.integers(-1, 2, y.size).astype(np.int32).reshape(y.shape)).view(np.float32)

    def run(rng):
        if rng is not None:
            def attn32(q, K16, V16, scale):
                q16 = R.f32_to_f16(q).astype(np.float32)
                s = ulp((K16.astype(np.float32) @ q16).astype(np.float32), rng)
                p16 = R.f32_to_f16(R.soft_max(s, scale)).astype(np.float32)
                return ulp((p16 @ V16.astype(np.float32)).astype(np.float32), rng)

            def mm(raw, t, K, x):
                if t == R.F32:   # F32 weights (the MoE router): an fp32 dot, as ggml_vec_dot_f32 forms it
                    W = np.ascontiguousarray(raw).view(np.float32).reshape(-1, K)
                    return ulp(W @ np.asarray(x, np.float32).reshape(-1), rng)
                return ulp(orig(raw, t, K, x), rng)
            R.mul_mat_vec = mm
            R.attention_head = attn32
        try:
            orc = oracle_from_gguf(buf, n_ctx=n_ctx)
            outs = [orc.decode(prompt).astype(np.float64)]
            outs += [orc.decode_one(t).astype(np.float64) for t in tokens]
        finally:
            R.mul_mat_vec = orig
            R.attention_head = orig_attn
        return outs

    base = run(None)
    floor = np.zeros(len(base))
    for r in range(runs):
        for i, o in enumerate(run(np.random.default_rng(seed + r))):
            floor[i] = max(floor[i], float(np.max(np.abs(o - base[i]))))
    return base, floor


def c_alt_floor(buf, n_ctx, prompt, tokens):
    """As oracle_ulp_floor, with the C oracle (LLaMA graphs) and one perturbation: the 8 float
    lanes of every k-quant dot summed in the reverse order (ORC_ALT).  Returns (base outputs,
    per-output max|alt - base|)."""
    import ggml_cpu
    a, b = ggml_cpu.Model(buf, n_ctx=n_ctx), ggml_cpu.Model(buf, n_ctx=n_ctx)
    try:
        base = [a.decode(prompt).astype(np.float64)]
        for t in prompt:
            alt = b.decode_one(t, alt=True)
        floor = [float(np.max(np.abs(alt - base[0])))]
        for t in tokens:
            base.append(a.decode_one(t).astype(np.float64))
            floor.append(float(np.max(np.abs(b.decode_one(t, alt=True) - base[-1]))))
    finally:
        a.close()
        b.close()
    return base, np.array(floor)


def parse_state(st: bytes, n_layer: int, kv_dim: int):
    """Split an mi_state_get() blob: (cell_pos, K[n_layer][n_cells][kv_dim], V[...])."""
    import struct
    st = np.frombuffer(st, np.uint8)
    h = struct.unpack("8s8i", st[:40].tobytes())
    nc = h[5]
    pos = np.frombuffer(st[40:40 + nc * 4].tobytes(), np.int32)
    off = 40 + nc * 4
    n = n_layer * nc * kv_dim * 2
    k = np.frombuffer(st[off:off + n].tobytes(), np.float16).reshape(n_layer, nc, kv_dim)
    v = np.frombuffer(st[off + n:off + 2 * n].tobytes(), np.float16).reshape(n_layer, nc, kv_dim)
    return pos, k, v


# A routing near-tie: the oracle's router separates the last expert picked from the first one left
# out by less than this (probability units); any other fp32 order may then pick the other expert.
ROUTE_TIE = 0.01
