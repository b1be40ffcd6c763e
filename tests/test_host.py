"""The bl::llama host surface (blama_amd/host, C++) through its C++ tests (tests/cpp/t_bl_llama.cpp),
which mirror inference/test/t-LogitComparer.cpp and t-integration.cpp.

CPU: LogitComparer KAT, sampler chain, vocab-only model and SPM tokenizer.
GPU: the session cases, then "compare - with model" (t-LogitComparer.cpp:41-79).  The GPU session
completes 12 tokens, and the CPU oracle verifies them the way Session::fillCtx does: at every
step it takes its logits at the claimed top-10 ids.  The result must pass the reference gate
(score >= 0.95, average similarity >= 0.98)."""
import os
import subprocess

import numpy as np
import pytest

import ggml_ref as R
from blama_amd import gguf, synthetic
from util import oracle_from_gguf

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "build", "t_bl_llama")
PROMPT = [1, 300, 301, 302, 303, 400, 77, 5]     # kPrompt in t_bl_llama.cpp


def _binary():
    if not os.path.exists(BIN):   # host-only g++ build (no HIP compile); build() normally did it
        subprocess.run(["make", "-C", os.path.join(ROOT, "blama_amd", "host")], check=True,
                       capture_output=True)
    return BIN


def vocab_gguf(path):
    """A small SentencePiece vocabulary with merges up to '▁hello' and '▁world'."""
    cfg = synthetic.CONFIGS["tiny-q4_k_m"]
    sp = "▁"
    pieces = [(sp, -20.0)] + [(c, -30.0) for c in "helowrd"] + [
        ("he", -1.0), ("ll", -2.0), ("llo", -3.0), ("hello", -4.0), (sp + "hello", -5.0),
        ("or", -6.0), ("ld", -7.0), ("wor", -8.0), ("world", -9.0), (sp + "world", -10.0)]
    toks = ["<unk>", "<s>", "</s>"] + ["<0x%02X>" % i for i in range(256)] + [p for p, _ in pieces]
    scores = [0.0, 0.0, 0.0] + [0.0] * 256 + [s for _, s in pieces]
    ttype = [2, 3, 3] + [6] * 256 + [1] * len(pieces)
    w = gguf.GGUFWriter()
    w.add_str("general.architecture", "llama")
    a = "llama"
    w.add_u32(f"{a}.context_length", cfg.n_ctx_train)
    w.add_u32(f"{a}.embedding_length", cfg.n_embd)
    w.add_u32(f"{a}.block_count", cfg.n_layer)
    w.add_u32(f"{a}.feed_forward_length", cfg.n_ff)
    w.add_u32(f"{a}.attention.head_count", cfg.n_head)
    w.add_u32(f"{a}.attention.head_count_kv", cfg.n_head_kv)
    w.add_f32(f"{a}.attention.layer_norm_rms_epsilon", cfg.eps)
    w.add_str("tokenizer.ggml.model", "llama")
    w.add_array("tokenizer.ggml.tokens", gguf.T_STRING, toks)
    w.add_array("tokenizer.ggml.scores", gguf.T_FLOAT32, scores)
    w.add_array("tokenizer.ggml.token_type", gguf.T_INT32, ttype)
    w.add_u32("tokenizer.ggml.bos_token_id", 1)
    w.add_u32("tokenizer.ggml.eos_token_id", 2)
    w.add_bool("tokenizer.ggml.add_bos_token", True)
    w.to_bytes().tofile(path)


def _run(args, timeout=240):
    r = subprocess.run([_binary()] + args, capture_output=True, text=True, timeout=timeout)
    print(r.stdout[-4000:], r.stderr[-2000:])
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    return r


def test_host_cpu_cases(tmp_path):
    v = str(tmp_path / "vocab.gguf")
    vocab_gguf(v)
    _run(["cpu", f"--vocab={v}"])


@pytest.mark.gpu
def test_host_gpu_sessions_and_compare_with_oracle(tmp_path):
    cfg = synthetic.CONFIGS["tiny-q4_k_m"]
    buf = synthetic.build_gguf(cfg, seed=11)
    mpath, out = str(tmp_path / "model.gguf"), str(tmp_path / "complete.txt")
    buf.tofile(mpath)
    _run(["gpu", f"--model={mpath}", f"--out={out}"])
    # "compare - with model": the CPU side verifies the GPU completion like Session::fillCtx
    preds = []
    for line in open(out):
        f = line.split()
        preds.append((int(f[0]), [(int(t.split(":")[0]), float(t.split(":")[1])) for t in f[1:]]))
    assert len(preds) == 12
    orc = oracle_from_gguf(buf, n_ctx=64)
    orc.decode(PROMPT)
    agg = R.MetricsAggregator()
    sims, score = [], None
    for tok, claimed in preds:
        # getToken records the top-10 AFTER decoding the sampled token (its getLogitsFromCtx
        # flushes the pending token first, Session.cpp:169-190, :252), as fillCtx does (:235-241)
        lg = orc.decode_one(tok)
        ids = sorted({i for i, _ in claimed})
        mine = sorted(R.gather(lg, ids), key=lambda t: -t[1])
        m = R.compare(claimed, mine)
        score = agg.push_and_verify([m])
        sims.append(R.logit_similarity(claimed, mine))
        assert m.top1Match == 1.0
    assert score >= 0.95 and float(np.mean(sims)) >= 0.98, (score, np.mean(sims))
