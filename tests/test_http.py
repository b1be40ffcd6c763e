"""blama-http-server (blama_amd/host/http_main.cpp) over real sockets, the way the reference's
server/code/http/test.rb drives the server: POST /complete, then POST /verify_completion with
that request and response.

CPU: env validation fails with the reference's messages (HttpServerMain.cpp:383-435), before any
GPU work.
GPU: a synthetic model served on 127.0.0.1.
  - /complete returns the wire format.
  - Verifying the completion with the server itself scores 1 (to fp32 order on the MFMA batch path).
  - A tampered completion scores lower.
  - The CPU oracle verifies the same HTTP completion like Session::fillCtx (score >= 0.95).
  - Non-POST gives 400, an unknown path 404, a malformed body 500."""
import json
import os
import re
import subprocess
import time
import urllib.error
import urllib.request

import numpy as np
import pytest

import ggml_ref as R
from blama_amd import synthetic
from util import oracle_from_gguf

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "blama_amd", "blama-http-server")


def _binary():
    if not os.path.exists(BIN):
        subprocess.run(["make", "-C", os.path.join(ROOT, "blama_amd", "host")], check=True,
                       capture_output=True)
    return BIN


def _run_env(env, timeout=30):
    e = dict(os.environ)
    for k in ("BLAMA_MODEL", "BLAMA_PORT", "BLAMA_HOST"):
        e.pop(k, None)
    e.update(env)
    return subprocess.run([_binary()], env=e, capture_output=True, text=True, timeout=timeout)


def test_env_validation(tmp_path):
    r = _run_env({})
    assert r.returncode == 1 and "Environment variable not set or empty: BLAMA_MODEL" in r.stderr
    r = _run_env({"BLAMA_MODEL": str(tmp_path / "m.bin")})
    assert "BLAMA_MODEL does not end with .gguf" in r.stderr
    r = _run_env({"BLAMA_MODEL": str(tmp_path / "missing.gguf")})
    assert "BLAMA_MODEL does not exist" in r.stderr
    (tmp_path / "d.gguf").mkdir()
    r = _run_env({"BLAMA_MODEL": str(tmp_path / "d.gguf")})
    assert "BLAMA_MODEL is not a regular file" in r.stderr
    r = _run_env({"BLAMA_PORT": "73x1"})
    assert "Extra characters after BLAMA_PORT number" in r.stderr
    r = _run_env({"BLAMA_PORT": "70000"})
    assert "Value exceeds uint16_t max" in r.stderr
    r = _run_env({"BLAMA_HOST": "not-an-address"})
    assert "Invalid BLAMA_HOST" in r.stderr


def _post(port, path, body, method="POST"):
    data = body.encode() if isinstance(body, str) else (json.dumps(body).encode() if body is not None else None)
    req = urllib.request.Request(f"http://127.0.0.1:{port}{path}", data=data, method=method)
    try:
        with urllib.request.urlopen(req, timeout=60) as r:
            return r.status, r.read().decode(), r.headers
    except urllib.error.HTTPError as e:
        return e.code, e.read().decode(), e.headers


def _prompt_ids(text):
    """Tokenisation of `text` by the synthetic vocabulary: BOS, then SPM's whitespace-escaped
    text as byte tokens (the vocabulary's only pieces are '▁t<n>', which never match)."""
    return [1] + [3 + b for b in ("▁" + text.replace(" ", "▁")).encode()]


def _piece(tid):
    """Vocab::tokenToString for the synthetic vocabulary (synthetic.vocab_tokens)."""
    if tid < 3:
        return {0: "\u2585", 1: "<s>", 2: "</s>"}[tid].encode()   # unknown prints U+2585
    if tid < 259:
        return bytes([tid - 3])
    return (" t%d" % (tid - 259)).encode()


@pytest.fixture
def served(tmp_path):
    yield from _serve(tmp_path, synthetic.CONFIGS["tiny-q4_k_m"])


def _start_server(env, log_dir, limit=300):
    """Start blama-http-server with stdout+stderr going to `log_dir`/server.log (a file, so a chatty
    server can never block on a full pipe) and wait for its "Listening on port" line.  If the
    server exits or the limit passes first, fail with its return code (negative = the signal
    that ended it) and everything it wrote: the stage log, RCCL's WARN lines, a backtrace."""
    log_path = os.path.join(str(log_dir), "server.log")
    log = open(log_path, "w")
    env = dict(env)
    env.setdefault("NCCL_DEBUG", "WARN")
    proc = subprocess.Popen([_binary()], env=env, stdout=log, stderr=subprocess.STDOUT)
    log.close()
    t0 = time.time()
    port, text = None, ""
    while time.time() - t0 < limit:
        with open(log_path, errors="replace") as f:
            text = f.read()
        m = re.search(r"^Listening on port (\d+)$", text, re.M)
        if m:
            port = int(m.group(1))
            break
        if proc.poll() is not None:
            break
        time.sleep(0.1)
    if not port:
        rc = proc.poll()
        if rc is None:
            proc.kill()      # the exact child we started
            proc.wait(timeout=30)
        with open(log_path, errors="replace") as f:
            text = f.read()
        raise AssertionError(f"server did not start (returncode {rc}, after {time.time() - t0:.1f} s); "
                             f"its output:\n{text[-6000:]}")
    return proc, port


def _stop_server(proc):
    proc.kill()              # the exact child we started
    proc.wait(timeout=30)


def _serve(tmp_path, cfg, devices=None):
    buf = synthetic.build_gguf(cfg, seed=5)
    path = str(tmp_path / "model.gguf")
    buf.tofile(path)
    env = dict(os.environ, BLAMA_MODEL=path, BLAMA_HOST="127.0.0.1", BLAMA_PORT="0")
    if devices:
        env["BLAMA_DEVICES"] = devices
    proc, port = _start_server(env, tmp_path)
    try:
        yield port, buf
    finally:
        _stop_server(proc)


@pytest.mark.gpu
def test_http_complete_and_verify(served):
    port, buf = served
    req = {"prompt": "hello world", "max_tokens": 10, "seed": 9, "temp": 0.8, "top_p": 0.95}
    st, body, hdr = _post(port, "/complete", req)
    assert st == 200, body
    assert hdr["Access-Control-Allow-Origin"] == "*"
    out = json.loads(body)
    toks = out["tokenData"]
    assert len(toks) == 10
    # token strings are raw vocabulary bytes; invalid UTF-8 is sent as U+FFFD (json.hpp)
    raw = [_piece(t["id"]) for t in toks]
    assert [t["str"] for t in toks] == [r.decode("utf-8", errors="replace") for r in raw]
    assert out["text"] == b"".join(raw).decode("utf-8", errors="replace")
    for t in toks:
        lg = [l["logit"] for l in t["logits"]]
        assert len(lg) == 10 and lg == sorted(lg, reverse=True)
    # self-verification through the wire format (Server.cpp:127-161).  The server pushes the
    # claimed tokens in one batched pass (mi_decode MI_OUT_ALL on the int8-MFMA GEMM for this
    # Q4_K_M model), whose rows match its own GEMV generation within fp32 summation order:
    # the score is 1 up to that (exactly 1 with BLAMA_SERIAL_VERIFY=1, the reference's loop)
    st, body, _ = _post(port, "/verify_completion", {"request": req, "response": out})
    assert st == 200, body
    assert json.loads(body)["result"] >= 0.999
    # tampered logits score lower
    bad = json.loads(json.dumps(out))
    for t in bad["tokenData"]:
        for l in t["logits"]:
            l["logit"] *= 1.5
    st, body, _ = _post(port, "/verify_completion", {"request": req, "response": bad})
    assert st == 200 and json.loads(body)["result"] < 0.95
    # the CPU oracle verifies the HTTP completion like fillCtx (t-LogitComparer.cpp:41-79 gate)
    orc = oracle_from_gguf(buf, n_ctx=64)
    orc.decode(_prompt_ids(req["prompt"]))
    agg = R.MetricsAggregator()
    sims, score = [], None
    for t in toks:
        claimed = [(l["id"], l["logit"]) for l in t["logits"]]
        lg = orc.decode_one(t["id"])
        mine = sorted(R.gather(lg, sorted({i for i, _ in claimed})), key=lambda x: -x[1])
        score = agg.push_and_verify([R.compare(claimed, mine)])
        sims.append(R.logit_similarity(claimed, mine))
    assert score >= 0.95 and float(np.mean(sims)) >= 0.98, (score, np.mean(sims))
    # protocol errors (HttpServerMain.cpp:305-309, :350-354)
    assert _post(port, "/complete", None, method="GET")[0] == 400
    assert _post(port, "/nowhere", req)[0] == 404
    assert _post(port, "/complete", "{not json")[0] == 500
    assert _post(port, "/complete", {"max_tokens": 3})[0] == 500          # "prompt" is required
    # the server keeps serving after errors
    st, body, _ = _post(port, "/complete", dict(req, max_tokens=2))
    assert st == 200 and len(json.loads(body)["tokenData"]) == 2


@pytest.fixture
def served_tinyllama(tmp_path):
    """BASELINE configs[0]: a TinyLlama-1.1B-shaped Q8_0 model (real width, heads 32/4,
    n_ff 5632, V 32000; 2 layers instead of 22 to bound the file)."""
    yield from _serve(tmp_path, synthetic.small_config("tinyllama-1.1b-q8_0", n_layer=2))


@pytest.mark.gpu
def test_http_tinyllama_complete_32_verified_by_oracle(served_tinyllama):
    """/complete of 32 tokens on the TinyLlama-shaped Q8_0 model, then the C restatement of the
    CPU path verifies the completion as Session::fillCtx would (Session.cpp:231-282) under the
    reference's gate (t-LogitComparer.cpp:76-78), and the server's own /verify_completion of it
    scores 1 to the fp32 order of the batched pass (Q8_0 batches run on the int8 MFMA GEMM
    with Q8_0 activations, as vec_dot_q8_0_q8_0)."""
    import ggml_cpu
    port, buf = served_tinyllama
    req = {"prompt": "the quick brown fox", "max_tokens": 32, "seed": 3, "temp": 0.8, "top_p": 0.95}
    st, body, _ = _post(port, "/complete", req)
    assert st == 200, body
    out = json.loads(body)
    toks = out["tokenData"]
    assert len(toks) == 32
    st, vbody, _ = _post(port, "/verify_completion", {"request": req, "response": out})
    assert st == 200 and json.loads(vbody)["result"] >= 0.999
    orc = ggml_cpu.Model(buf, n_ctx=128)
    orc.decode(_prompt_ids(req["prompt"]))
    agg = R.MetricsAggregator()
    sims, top1, score = [], [], None
    for t in toks:
        claimed = [(l["id"], l["logit"]) for l in t["logits"]]
        lg = orc.decode_one(t["id"])
        mine = sorted(R.gather(lg, sorted({i for i, _ in claimed})), key=lambda x: -x[1])
        cm = R.compare(claimed, mine)
        top1.append(cm.top1Match)
        score = agg.push_and_verify([cm])
        sims.append(R.logit_similarity(claimed, mine))
    orc.close()
    assert score >= 0.95 and float(np.mean(sims)) >= 0.98 and min(top1) == 1.0, (score, np.mean(sims))


@pytest.fixture
def served_replicas(tmp_path):
    # configs[3]'s shape at small scale: 4 replicas (one Model + Instance + worker each) behind
    # the least-loaded dispatcher; on the 8-GPU node BLAMA_DEVICES=0,...,7 puts one per GPU
    yield from _serve(tmp_path, synthetic.CONFIGS["tiny-q4_k_m"], devices="0,0,0,0")


@pytest.mark.gpu
def test_http_concurrent_verify_on_replicas(served_replicas):
    """8 concurrent /verify_completion requests (BASELINE configs[3] is 8 concurrent sessions on
    8 GPUs) against a server with 4 replicas: every request is answered, each completion
    verifies itself (score >= 0.999 through the batched pass), and a tampered one scores low."""
    import threading
    port, _ = served_replicas
    reqs = [{"prompt": f"request number {i}", "max_tokens": 12, "seed": i, "temp": 0.8, "top_p": 0.95}
            for i in range(8)]
    outs = [None] * 8

    def complete(i):
        st, body, _ = _post(port, "/complete", reqs[i])
        assert st == 200, body
        outs[i] = json.loads(body)

    th = [threading.Thread(target=complete, args=(i,)) for i in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert all(o is not None and len(o["tokenData"]) == 12 for o in outs)
    results = [None] * 8

    def verify(i):
        body = {"request": reqs[i], "response": outs[i]}
        if i == 7:   # one tampered completion
            body = json.loads(json.dumps(body))
            for t in body["response"]["tokenData"]:
                for l in t["logits"]:
                    l["logit"] *= 1.5
        st, rb, _ = _post(port, "/verify_completion", body)
        assert st == 200, rb
        results[i] = json.loads(rb)["result"]

    th = [threading.Thread(target=verify, args=(i,)) for i in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert all(r is not None and r >= 0.999 for r in results[:7]), results
    assert results[7] < 0.95


@pytest.fixture(scope="module")
def llama3_bpe_model(tmp_path_factory):
    """BASELINE configs[3]'s model at full width: Llama-3-8B Q6_K shape (n_embd 4096, heads
    32/8, n_ff 14336, V = 128256; 2 layers instead of 32 to bound the file) with a byte-level
    BPE ("gpt2") vocabulary of 128256 entries, so prompts go through the BPE tokenizer."""
    cfg = synthetic.small_config("llama3-8b-q6_k", n_layer=2)
    vocab = synthetic.bpe_vocab(cfg.n_vocab)
    buf = synthetic.build_gguf(cfg, seed=7, vocab=vocab)
    path = str(tmp_path_factory.mktemp("l3") / "llama3.gguf")
    buf.tofile(path)
    return cfg, vocab, buf, path


def _serve_path(path, env_extra):
    env = dict(os.environ, BLAMA_MODEL=path, BLAMA_HOST="127.0.0.1", BLAMA_PORT="0", **env_extra)
    return _start_server(env, os.path.dirname(path))


@pytest.mark.gpu
def test_http_llama3_width_concurrent_verify_on_replicas(llama3_bpe_model):
    """configs[3] at its shape on one GPU: Llama-3-8B width, BPE vocabulary, 4 replicas
    (BLAMA_DEVICES=0,0,0,0; replica 1 receives the weight arena through a one-rank RCCL
    broadcast, MI_REPLICATE_RCCL=1, replicas 2-3 by device copies -- none re-reads the GGUF's
    tensor data), 8 concurrent /complete then 8 concurrent /verify_completion:
      * every completion self-verifies (score >= 0.999 through the batched pass);
      * one tampered completion scores < 0.95;
      * the C restatement of the CPU path verifies every completion as Session::fillCtx would
        (Session.cpp:231-282), each under the reference gate (t-LogitComparer.cpp:76-78)."""
    import threading
    import ggml_cpu
    cfg, vocab, buf, path = llama3_bpe_model
    proc, port = _serve_path(path, {"BLAMA_DEVICES": "0,0,0,0", "MI_REPLICATE_RCCL": "1"})
    try:
        reqs = [{"prompt": f"request number {i}: the quick brown fox", "max_tokens": 10, "seed": 100 + i,
                 "temp": 0.8, "top_p": 0.95} for i in range(8)]
        outs = [None] * 8

        def complete(i):
            st, body, _ = _post(port, "/complete", reqs[i])
            assert st == 200, body
            outs[i] = json.loads(body)

        th = [threading.Thread(target=complete, args=(i,)) for i in range(8)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=300)
        assert all(o is not None and len(o["tokenData"]) == 10 for o in outs), outs
        # the wire's token strings are the BPE vocabulary's pieces, decoded from byte-level form
        tk = vocab["tokenizer"]
        for o in outs:
            for t in o["tokenData"]:
                if vocab["types"][t["id"]] == 1:
                    assert t["str"] == tk.decode([t["id"]]), t
        results = [None] * 8

        def verify(i):
            body = {"request": reqs[i], "response": outs[i]}
            if i == 7:
                body = json.loads(json.dumps(body))
                for t in body["response"]["tokenData"]:
                    for l in t["logits"]:
                        l["logit"] *= 1.5
            st, rb, _ = _post(port, "/verify_completion", body)
            assert st == 200, rb
            results[i] = json.loads(rb)["result"]

        th = [threading.Thread(target=verify, args=(i,)) for i in range(8)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=300)
        assert all(r is not None and r >= 0.999 for r in results[:7]), results
        assert results[7] < 0.95, results
    finally:
        _stop_server(proc)
    # the CPU oracle verifies each completion on its own session (prompt: BOS + BPE ids)
    orc = ggml_cpu.Model(buf, n_ctx=64)
    try:
        for i in range(8):
            orc.reset()
            orc.decode([vocab["bos"]] + tk.encode(reqs[i]["prompt"], add_special_tokens=False).ids)
            agg = R.MetricsAggregator()
            sims, top1, score = [], [], None
            for t in outs[i]["tokenData"]:
                claimed = [(l["id"], l["logit"]) for l in t["logits"]]
                lg = orc.decode_one(t["id"])
                mine = sorted(R.gather(lg, sorted({x for x, _ in claimed})), key=lambda x: -x[1])
                cm = R.compare(claimed, mine)
                top1.append(cm.top1Match)
                score = agg.push_and_verify([cm])
                sims.append(R.logit_similarity(claimed, mine))
            assert score >= 0.95 and float(np.mean(sims)) >= 0.98 and min(top1) == 1.0, (i, score, np.mean(sims))
    finally:
        orc.close()
