"""csv_shard: reference goldens + byte-for-byte parity with csv.DictReader."""
import csv
import io
import os

import pytest

from ops.csv_shard import read_shard


@pytest.fixture()
def ten_rows(tmp_path):
    p = tmp_path / "t.csv"
    p.write_text("id,text,risk\n" + "".join(f"{i},row {i},{i / 10}\n" for i in range(10)))
    return str(p)


def test_goldens(ten_rows):
    F = ten_rows
    out = read_shard({"source_uri": F, "start_row": 2, "shard_size": 3, "dataset_id": "d"})
    assert out == {"ok": True, "dataset_id": "d", "mode": "rows", "start_row": 2, "end_row": 5, "row_count": 3,
                   "rows": [{"id": "2", "text": "row 2", "risk": "0.2"}, {"id": "3", "text": "row 3", "risk": "0.3"},
                            {"id": "4", "text": "row 4", "risk": "0.4"}]}
    assert read_shard({"payload": {"source_uri": F, "start_row": 8, "shard_size": 5, "mode": "count"}}) == {
        "ok": True, "dataset_id": "unknown_dataset", "mode": "count", "start_row": 8, "end_row": 10, "row_count": 2}


@pytest.mark.parametrize("payload,err", [
    (None, "read_csv_shard: missing payload"),
    ([1], "read_csv_shard: payload must be a dict"),
    ({"x": 1}, "read_csv_shard: payload.source_uri (string) is required"),
    ({"source_uri": "/nope"}, "read_csv_shard: file not found: /nope"),
    ({"source_uri": "F", "start_row": -1}, "read_csv_shard: start_row must be >= 0"),
    ({"source_uri": "F", "shard_size": 0}, "read_csv_shard: shard_size must be > 0"),
    ({"source_uri": "F", "mode": "x"}, "read_csv_shard: mode must be 'rows' or 'count'"),
    ({"source_uri": "F", "start_row": "a"}, "read_csv_shard: start_row and shard_size must be integers"),
    ({"payload": None}, "read_csv_shard: payload must be a dict"),
])
def test_errors(ten_rows, payload, err):
    if isinstance(payload, dict) and payload.get("source_uri") == "F":
        payload = dict(payload, source_uri=ten_rows)
    assert read_shard(payload) == {"ok": False, "error": err}


TRICKY = [
    'a,b,c\n1,2,3\n',
    'a,b,c\r\n1,2,3\r\n4,5,6',                       # CRLF, no trailing newline
    'a,b\n"x, y","he said ""hi"""\n',                  # quotes, escaped quotes
    'a,b\n"multi\nline",2\n"cr\r\nlf",3\n',           # newlines inside quotes
    'a,b\n\n\n1,2\n\r\n3,4\n',                         # blank lines skipped
    'a,b,c\n1\n1,2,3,4,5\n',                          # short and long rows
    'a,b\n"ab"cd,2\nx"y,3\n',                          # text after closing quote; literal quote
    'a,a,b\n1,2,3\n',                                   # duplicate header: last wins
    '﻿id,text\n1,naïve café 東京\n',                # BOM + unicode
    'a,b\n1,"unterminated\n2,3\n',                     # unterminated quote runs to EOF
    'a,b\n,\n"",""\n',                                  # empty fields
    'x\n1\r2\r3\n',                                     # lone CR terminators
    '\n\nh1,h2\n1,2\n',                                 # leading blank line -> fieldnames []
]


@pytest.mark.parametrize("text", TRICKY)
def test_parity_with_dictreader(tmp_path, text):
    p = tmp_path / "x.csv"
    p.write_bytes(text.encode("utf-8"))
    with open(p, newline="", encoding="utf-8") as f:
        ref = list(csv.DictReader(f))
    got = read_shard({"source_uri": str(p), "start_row": 0, "shard_size": 1000})
    assert got["ok"] and got["rows"] == ref
    for s in range(len(ref)):
        assert read_shard({"source_uri": str(p), "start_row": s, "shard_size": 2})["rows"] == ref[s:s + 2]


def test_deep_offset_and_cache(tmp_path):
    from agent_tpu_amd.utils.synthetic import write_csv

    p = write_csv(str(tmp_path / "big.csv"), 5000, words_per_row=8, seed=2)
    with open(p, newline="", encoding="utf-8") as f:
        ref = list(csv.DictReader(f))
    out = read_shard({"source_uri": p, "start_row": 4990, "shard_size": 100})
    assert len(ref) == 5000
    assert out["row_count"] == 10 and out["rows"] == ref[4990:]
    from agent_tpu_amd.io.csv import open_csv

    assert open_csv(p) is open_csv(p)  # index built once per file version


def test_native_column_extract_and_floats(tmp_path, nat):
    from agent_tpu_amd.utils.synthetic import write_csv

    p = write_csv(str(tmp_path / "c.csv"), 300, words_per_row=5, seed=4)
    with open(p, newline="", encoding="utf-8") as f:
        ref = list(csv.DictReader(f))
    t = nat.CsvTable(p)
    text, offs = t.extract_column(10, 50, t.column_index("text"), 4096, 4)
    blob = text.tobytes()
    got = [blob[offs[i]:offs[i + 1]].decode() for i in range(50)]
    assert got == [r["text"] for r in ref[10:60]]
    vals = t.float_column(0, 300, t.column_index("risk"), 4)
    assert list(vals) == [float(r["risk"]) for r in ref]
    with pytest.raises(ValueError, match="could not convert string to float"):
        t.float_column(0, 5, t.column_index("text"), 1)


def test_persisted_row_index(tmp_path, monkeypatch):
    """ATPU_CSV_INDEX_DIR persists the row index; a changed file invalidates it."""
    import os
    import subprocess
    import sys

    from agent_tpu_amd.utils.synthetic import write_csv

    path = str(tmp_path / "big.csv")
    write_csv(path, 2000, 20)
    idx_dir = tmp_path / "idx"
    idx_dir.mkdir()
    code = ("import sys; sys.path.insert(0, %r); import torch; from agent_tpu_amd._native import native; "
            "t = native().CsvTable(%r); print(t.index_from_cache, t.num_rows, t.row(1234)[0])") % (
        os.getcwd(), path)
    env = dict(os.environ, ATPU_CSV_INDEX_DIR=str(idx_dir))
    run = lambda: subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,  # noqa: E731
                                 timeout=120).stdout.split()
    first, second = run(), run()
    assert first[0] == "False" and second[0] == "True" and first[1:] == second[1:] == ["2000", "1234"]
    assert len(list(idx_dir.iterdir())) == 1
    with open(path, "a") as f:
        f.write("2000,new row,0.5\n")
    third = run()
    assert third[0] == "False" and third[1] == "2001"
