"""The C-ABI library loads on a CPU-only host and exports every symbol the
public header declares (no compute is called without a GPU)."""
import ctypes
import os

from blama_amd import engine


def test_library_exists_and_loads():
    assert os.path.exists(engine.LIB_PATH), "run __graft_entry__.build() first"
    L = engine.lib()
    assert L is not None


def test_header_symbols_exported():
    syms = engine.header_symbols()
    assert len(syms) >= 40
    L = ctypes.CDLL(engine.LIB_PATH)
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing


def test_binding_covers_header():
    assert set(engine.header_symbols()) == set(engine._SIGS)


def test_vocab_only_load_needs_no_gpu():
    """Model::Params{.vocabOnly=true} parses metadata + vocab only (t-integration.cpp:25-43)."""
    from blama_amd import synthetic
    buf = synthetic.build_gguf(synthetic.CONFIGS["tiny-q8_0"])
    m = engine.Model(buf, vocab_only=True)
    assert m.n_vocab == 384 and m.n_embd == 256 and m.n_ctx_train == 256
    assert m.token_text(1) == "<s>" and m.token_text(2) == "</s>"
    assert m.bos == 1 and m.eos == 2 and m.is_eog(2) and not m.is_eog(5)


def test_errors_are_reported_not_thrown():
    import pytest
    with pytest.raises(engine.EngineError, match="not a GGUF"):
        engine.Model(b"NOPE" + bytes(64), vocab_only=True)
    with pytest.raises(engine.EngineError, match="cannot open"):
        engine.Model("/nonexistent/model.gguf")
