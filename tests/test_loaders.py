"""On-disk formats either side of the path, CPU only:
  * the llama2.c v0 fp32 model.bin reader (read_checkpoint, reference src/utils.cpp:150-170);
  * the runq v2 "ak42" int8 reader (thallama_q8_read_checkpoint, runq.c:219-251).
Files are written by the oracle (oracle.c write_v0 / write_v2, the export.py layouts pinned in
tests/test_oracle.py against the reference's own runq.c reader); the readers must hand back
the exact bytes."""
import ctypes as C

import numpy as np
import pytest

from helpers import SMALL, SMALL_GQA


@pytest.mark.parametrize("cfg,shared", [(SMALL, 0), (SMALL, 1), (SMALL_GQA, 0)])
def test_v0_reader_maps_the_file(tl, oracle, tmp_path, cfg, shared):
    m = oracle.Model(cfg, shared, seed=12)
    path = str(tmp_path / "model.bin")
    m.write_v0(path)
    c, w = tl.Config(), tl.TransformerWeights()
    fd, data, size = C.c_int(-1), tl.c_float_p(), C.c_ssize_t(0)
    tl.lib().read_checkpoint(path.encode(), C.byref(c), C.byref(w), C.byref(fd), C.byref(data), C.byref(size))
    assert (c.dim, c.hidden_dim, c.n_layers, c.n_heads, c.n_kv_heads, c.vocab_size, c.seq_len) == \
        tuple(abs(v) for v in cfg)
    n = tl.lib().thallama_v0_payload_floats(C.byref(c), shared)
    got = np.ctypeslib.as_array(w.token_embedding_table, shape=(n,))
    np.testing.assert_array_equal(got, m.arena()[:n])
    # the classifier is the embedding iff the file says shared (positive vocab_size)
    assert (C.addressof(w.wcls.contents) == C.addressof(w.token_embedding_table.contents)) == bool(shared)


@pytest.mark.parametrize("cfg,shared,gs", [(SMALL, 0, 64), (SMALL, 1, 32), (SMALL_GQA, 0, 128)])
def test_v2_reader_returns_the_payload(tl, oracle, tmp_path, cfg, shared, gs):
    m = oracle.Model(cfg, shared, seed=3)
    m.build_q8(gs)
    path = str(tmp_path / "model_q8.bin")
    m.write_v2(path)
    ck = tl.Q8Checkpoint()
    assert tl.lib().thallama_q8_read_checkpoint(path.encode(), C.byref(ck)) == 0
    try:
        c = ck.config
        assert (c.dim, c.hidden_dim, c.n_layers, c.n_heads, c.n_kv_heads, c.vocab_size, c.seq_len) == cfg
        assert ck.shared_classifier == shared and ck.group_size == gs
        n = tl.lib().thallama_q8_payload_bytes(C.byref(c), shared, gs)
        assert ck.payload_bytes >= n
        got = np.ctypeslib.as_array(C.cast(ck.payload, C.POINTER(C.c_uint8)), shape=(n,))
        np.testing.assert_array_equal(got, m.q8_payload())
    finally:
        tl.lib().thallama_q8_close_checkpoint(C.byref(ck))


def test_v2_reader_errors(tl, oracle, tmp_path):
    ck = tl.Q8Checkpoint()
    assert tl.lib().thallama_q8_read_checkpoint(str(tmp_path / "missing.bin").encode(), C.byref(ck)) == -1
    m = oracle.Model(SMALL, 0, seed=3)
    m.build_q8(64)
    good = tmp_path / "good.bin"
    m.write_v2(str(good))
    raw = bytearray(good.read_bytes())
    bad = tmp_path / "bad.bin"
    bad.write_bytes(b"xxxx" + raw[4:])
    assert tl.lib().thallama_q8_read_checkpoint(str(bad).encode(), C.byref(ck)) == -2
    v3 = bytearray(raw)
    v3[4] = 3
    bad.write_bytes(bytes(v3))
    assert tl.lib().thallama_q8_read_checkpoint(str(bad).encode(), C.byref(ck)) == -3
    bad.write_bytes(bytes(raw[: len(raw) // 2]))
    assert tl.lib().thallama_q8_read_checkpoint(str(bad).encode(), C.byref(ck)) == -4
