"""DP collectives through a real RCCL communicator (world size 1, SURVEY.md
§4.4(4c)): backend "nccl" on ROCm. C1 weight broadcast of a ParamPack, C2
ragged all-gather, C3 risk all-reduce and C4 task descriptor run through
torch.distributed exactly as under torchrun, on cuda tensors."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SCRIPT = r'''
import os, sys, json
sys.path.insert(0, os.environ["REPO"])
import torch, torch.distributed as dist
from agent_tpu_amd.parallel import dp, dp_ops
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
assert dist.get_backend() == "nccl"
out = {}
from agent_tpu_amd.models.bert import config_for, init_random
cfg = config_for("bert-tiny")
pack = dp.broadcast_pack(init_random(cfg, seed=1), cfg, dev)
out["pack_on_gpu"] = pack.buffer.is_cuda and torch.equal(pack.buffer.cpu(), init_random(cfg, seed=1).buffer)
idx = torch.arange(37, dtype=torch.int32, device=dev).view(-1, 1).repeat(1, 2)
g, = dp.all_gather_rows(idx)
out["gather"] = g.is_cuda and torch.equal(g.cpu(), idx.cpu())
out["desc"] = dp.broadcast_task({"op": "x"}) == {"op": "x"}
vals = [float(i) / 7 for i in range(1000)]
r = dp_ops.dispatch("risk_accumulate", {"values": vals})
out["risk"] = r["count"] == 1000 and abs(r["sum"] - sum(vals)) < 1e-9 and r["dp_world_size"] == 1
from agent_tpu_amd.parallel import rccl
out["native"] = rccl.enabled() == (os.environ.get("ATPU_COMM") == "native") and (
    dp.native_comm(dev) is not None) == rccl.enabled()
if rccl.enabled():
    nc = dp.native_comm(dev)
    t = torch.arange(10, dtype=torch.float64, device=dev)
    nc.all_reduce(t, "max")
    b = torch.full((5,), 3, dtype=torch.bfloat16, device=dev)
    nc.broadcast(b, 0)
    o = torch.empty(5, dtype=torch.bfloat16, device=dev)
    nc.all_gather_into(o, b)
    out["native_ops"] = torch.equal(t.cpu(), torch.arange(10, dtype=torch.float64)) and torch.equal(o.cpu(), b.cpu()) and nc.healthy()
    # single-process form over the local GPU(s) (ncclCommInitAll)
    cs = rccl.local_comms([0])
    x = torch.ones(4, device=dev)
    with rccl.group():
        cs[0].all_reduce(x, "sum")
    torch.cuda.synchronize()
    out["init_all"] = cs[0].world == 1 and torch.equal(x.cpu(), torch.ones(4))
dist.barrier()
dist.destroy_process_group()
print("RESULT " + json.dumps(out))
'''


@pytest.mark.parametrize("comm", ["torch", "native"])
def test_rccl_world1_collectives(gpu, comm):
    """Same collectives through ProcessGroupNCCL and through the native RcclComm
    (ATPU_COMM=native: csrc/comm/rccl_comm.cpp)."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0", REPO=REPO, HSA_ENABLE_IPC_MODE_LEGACY="0", ATPU_COMM=comm)
    p = subprocess.run([sys.executable, "-c", SCRIPT], env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-3000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("RESULT ")][-1]
    import json

    res = json.loads(line[7:])
    want = {"pack_on_gpu": True, "gather": True, "desc": True, "risk": True, "native": True}
    if comm == "native":
        want.update(native_ops=True, init_all=True)
    assert res == want, res
