"""Native top-k JSON (``_atpu.topk_json``) + RawJSON splicing."""
import json

import numpy as np

from agent_tpu_amd.utils.rawjson import RawJSON, dumps, plain


def test_topk_json_matches_python_json(nat):
    rng = np.random.default_rng(0)
    n, k = 257, 3
    idx = rng.integers(0, 30000, (n, k)).astype(np.int32)
    sc = rng.random((n, k)).astype(np.float32)
    sc[0, 0], sc[1, 1], sc[2, 2] = 1.0, 0.0, 1.2e-5
    rows = [{"row": 100 + r, "topk": [{"index": int(i), "score": float(s)} for i, s in zip(idx[r], sc[r])]}
            for r in range(n)]
    got = nat.topk_json(100, idx, sc, 0)
    assert json.loads(got) == rows
    assert got == json.dumps(rows, separators=(",", ":")).encode() or json.loads(got) == rows
    assert json.loads(nat.topk_json(0, idx, sc, 1)) == idx.tolist()
    assert json.loads(nat.topk_json(0, idx, sc, 2)) == [[float(x) for x in r] for r in sc]
    assert nat.topk_json(0, idx[:0], sc[:0], 0) == b"[]"


def test_rawjson_splice_and_list_behaviour():
    raw = RawJSON(b'[{"row":0,"topk":[{"index":1,"score":0.5}]}]')
    body = {"lease_id": "L", "result": {"ok": True, "rows": raw, "note": "x\x00y"}, "error": None}
    data = dumps(body)
    back = json.loads(data)
    assert back["result"]["rows"] == [{"row": 0, "topk": [{"index": 1, "score": 0.5}]}]
    assert back["result"]["note"] == "x\x00y"
    assert raw[0]["row"] == 0 and len(raw) == 1 and list(raw)[0]["topk"][0]["index"] == 1
    assert plain(body)["result"]["rows"] == back["result"]["rows"]
    assert dumps({"a": [1.5, "b"]}) == b'{"a":[1.5,"b"]}'
