"""Byte-level BPE tokenisation (tokenizer.ggml.model "gpt2": Llama-3 and GPT-2 vocabularies),
reference Vocab::tokenize -> llama_tokenize (/root/reference/inference/code/llama/Vocab.cpp:37-51).

Parity: no Llama-3 tokenizer file or fixture ships with the reference, so the exact Llama-3 ids
are unpinned.  The algorithm is pinned instead against HuggingFace `tokenizers` (the library
that defines Llama-3's tokenizer.json: Split(regex, isolated) + ByteLevel(no prefix space,
no regex) + BPE(ignore_merges)) on a vocabulary trained here, and the pre-tokenizer alone
against the `regex` module running the Llama-3 / GPT-2 patterns of llama.cpp's
llama-vocab.cpp.  The C++ side is the host mirror's Vocab (blama_amd/host/llama.cpp) on a
vocab-only GGUF carrying that vocabulary and its merges."""
import os
import subprocess

import numpy as np
import pytest
import regex

from blama_amd import gguf, synthetic

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "build", "t_bl_llama")

LLAMA3 = (r"(?:'[sS]|'[tT]|'[rR][eE]|'[vV][eE]|'[mM]|'[lL][lL]|'[dD])|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}{1,3}|"
          r" ?[^\s\p{L}\p{N}]+[\r\n]*|\s*[\r\n]+|\s+(?!\S)|\s+")
GPT2 = r"'s|'t|'re|'ve|'m|'ll|'d| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+"

CORPUS = [
    "Hello world! It's a test, isn't it? We'll see: 12345 apples and 3.14159 pies.",
    "The quick brown fox jumps over the lazy dog.\n\nNew paragraph\twith\ttabs   and  spaces.",
    "Ünïcödé wörds, naïve café, résumé — em-dash… «quotes» and 日本語のテキスト、中文字符。",
    "Code: def f(x):\n    return x**2 + 1  # comment\r\nprint(f(3))",
    "I'M SHOUTING, YOU'RE QUIET, THEY'VE GONE, WE'D STAY, SHE'LL GO'S",
    "numbers 1 22 333 4444 55555 666666 and ٣٤٥ and ⅷ and ①②③",
    "emoji 🙂🚀 mixed with text🙂word and   \n  \n trailing   ",
]
TEXTS = CORPUS + [
    "", " ", "\n", "  leading", "trailing  ", "a\r\n\r\nb", "'s'S'll'LL", "x'y", "  \n\t  x",
    "hello<|special|>world", "<|special|>", "a <|special|> b",
    "ÀÁÂ123abc!!!???...", "tab\tsep\tvalues\t", " nbsp emsp　ideographic",
]


def _train(pre_pattern):
    from tokenizers import Regex, Tokenizer, decoders, models, pre_tokenizers, trainers
    tok = Tokenizer(models.BPE(ignore_merges=pre_pattern == LLAMA3))
    tok.pre_tokenizer = pre_tokenizers.Sequence([
        pre_tokenizers.Split(Regex(pre_pattern), behavior="isolated", invert=False),
        pre_tokenizers.ByteLevel(add_prefix_space=False, trim_offsets=False, use_regex=False)])
    tok.decoder = decoders.ByteLevel()
    trainer = trainers.BpeTrainer(vocab_size=600, min_frequency=1, special_tokens=["<|special|>"],
                                  initial_alphabet=pre_tokenizers.ByteLevel.alphabet(), show_progress=False)
    tok.train_from_iterator(CORPUS * 20, trainer=trainer)
    return tok


def _vocab_gguf(path, tok, pre):
    import json
    model = json.loads(tok.to_str())["model"]
    vocab = model["vocab"]
    merges = [m if isinstance(m, str) else " ".join(m) for m in model["merges"]]
    toks = [None] * len(vocab)
    for t, i in vocab.items():
        toks[i] = t
    ttype = [3 if t == "<|special|>" else 1 for t in toks]
    cfg = synthetic.CONFIGS["tiny-q4_k_m"]
    w = gguf.GGUFWriter()
    a = "llama"
    w.add_str("general.architecture", a)
    w.add_u32(f"{a}.context_length", cfg.n_ctx_train)
    w.add_u32(f"{a}.embedding_length", cfg.n_embd)
    w.add_u32(f"{a}.block_count", cfg.n_layer)
    w.add_u32(f"{a}.feed_forward_length", cfg.n_ff)
    w.add_u32(f"{a}.attention.head_count", cfg.n_head)
    w.add_u32(f"{a}.attention.head_count_kv", cfg.n_head_kv)
    w.add_f32(f"{a}.attention.layer_norm_rms_epsilon", cfg.eps)
    w.add_str("tokenizer.ggml.model", "gpt2")
    w.add_str("tokenizer.ggml.pre", pre)
    w.add_array("tokenizer.ggml.tokens", gguf.T_STRING, toks)
    w.add_array("tokenizer.ggml.token_type", gguf.T_INT32, ttype)
    w.add_array("tokenizer.ggml.merges", gguf.T_STRING, merges)
    w.add_u32("tokenizer.ggml.bos_token_id", 0)
    w.add_u32("tokenizer.ggml.eos_token_id", 0)
    w.to_bytes().tofile(path)


def _cxx_tokenize(vocab_path, texts, tmp_path):
    src, dst = tmp_path / "in.txt", tmp_path / "out.txt"
    src.write_text("\n".join(t.encode("utf-8").hex() for t in texts) + "\n")
    r = subprocess.run([BIN, "tok", f"--vocab={vocab_path}", f"--in={src}", f"--out={dst}"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = dst.read_text().split("\n")[:len(texts)]
    return [[int(x) for x in ln.split()] for ln in lines]


def _random_texts(n, seed):
    rng = np.random.default_rng(seed)
    alphabet = list("abcXYZ019 '\n\r\t.,!?-_()") + ["é", "ß", "日", "本", "🙂", " ", "٣", "Ω", "'s", "'LL"]
    return ["".join(rng.choice(alphabet, size=int(rng.integers(1, 40)))) for _ in range(n)]


@pytest.mark.parametrize("pattern,pre", [(LLAMA3, "llama-bpe"), (GPT2, "gpt-2")])
def test_bpe_matches_hf_tokenizers(tmp_path, pattern, pre):
    if not os.path.exists(BIN):
        subprocess.run(["make", "-C", os.path.join(ROOT, "blama_amd", "host")], check=True, timeout=600)
    tok = _train(pattern)
    vp = str(tmp_path / "bpe.gguf")
    _vocab_gguf(vp, tok, pre)
    texts = TEXTS + _random_texts(200, 3)
    got = _cxx_tokenize(vp, texts, tmp_path)
    for t, ids in zip(texts, got):
        want = tok.encode(t, add_special_tokens=False).ids
        assert ids == want, (t, ids, want)


@pytest.mark.parametrize("pattern", [LLAMA3, GPT2])
def test_pretokenizer_pattern_oracle(pattern):
    """The regex module's split is what HF's Split(isolated) produces; the C++ matcher is
    checked through the full encode above, this pins the patterns themselves."""
    for t in TEXTS:
        parts = regex.findall(pattern, t)
        assert "".join(parts) == t
