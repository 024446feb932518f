"""Hash-WordPiece spec "atpu-hash-wordpiece v1": the Python reference and the
C++ host twin agree byte for byte (the HIP kernel is pinned against both in
tests/kernels/test_kernels_gpu.py)."""
import numpy as np
import pytest

from agent_tpu_amd import tokenizer as T

ROWS = ["", "   ", "Hello, World!", "a" * 200, "ünïcödé wörds and émojis 🙂🙂 ok", "tab\tsep\nnew line",
        "x,y;z!?(paren) [br] {c}", "MiXeD CaSe 123 4567 89.01", "supercalifragilisticexpialidocious" * 3,
        "\x00\x01 control chars \x7f", " ".join(["tok"] * 300)]


@pytest.mark.parametrize("seq_len,vocab", [(128, 30522), (16, 32128), (512, 4096)])
def test_python_and_host_twins_agree(nat, seq_len, vocab):
    rows = [r.encode("utf-8") for r in ROWS]
    ids_py, lens_py = T.tokenize_rows(rows, seq_len, vocab)
    text, offs = T.pack_rows(rows)
    ids_h, lens_h = nat.tokenize_host(text, offs, seq_len, vocab, T.DEFAULT_MAX_ROW_BYTES)
    assert np.array_equal(np.asarray(lens_h), lens_py)
    assert np.array_equal(np.asarray(ids_h), ids_py)
    assert (ids_py[:, 0] == T.CLS_ID).all()
    assert all(ids_py[r, lens_py[r] - 1] == T.SEP_ID for r in range(len(rows)))
    assert ((ids_py == 0) | (ids_py == T.CLS_ID) | (ids_py == T.SEP_ID) | (ids_py >= 1000)).all()
    assert (ids_py < vocab).all()


def test_deterministic_and_case_insensitive():
    a = T.token_ids(b"Hello World", 30522, 64)
    assert a == T.token_ids(b"hello world", 30522, 64) == T.token_ids(b"HELLO   WORLD", 30522, 64)
    assert len(a) >= 2
