import sys, time, torch
sys.path.insert(0, "/root/repo")
import agent_tpu_amd.runtime.summarize as sm
from agent_tpu_amd.utils.synthetic import make_text_rows
T = {"cap": 0.0, "n": 0}
cb, ce = torch.cuda.CUDAGraph.capture_begin, torch.cuda.CUDAGraph.capture_end
def b(self, *a, **k):
    torch.cuda.synchronize(); T["t"] = time.perf_counter(); return cb(self, *a, **k)
def e(self, *a, **k):
    r = ce(self, *a, **k); torch.cuda.synchronize(); T["cap"] += time.perf_counter() - T["t"]; T["n"] += 1; return r
torch.cuda.CUDAGraph.capture_begin, torch.cuda.CUDAGraph.capture_end = b, e
for name in ("t5-base", "bart-large-cnn"):
    model, _ = sm.build_model(name, device=torch.device("cuda", 0), seed=0)
    eng = sm.SummarizeEngine(model, 512)
    gen = sm.GenConfig(num_beams=4, max_length=130, min_length=30)
    docs = make_text_rows(512, words_per_row=409, seed=5)
    eng.summarize(docs[:256], gen); torch.cuda.synchronize()
    T.update(cap=0.0, n=0)
    t = time.perf_counter(); eng.summarize(docs[256:], gen); torch.cuda.synchronize(); wall = time.perf_counter() - t
    print(f"{name}: wall {wall*1e3:.0f} ms, graph capture+instantiate {T['cap']*1e3:.1f} ms over {T['n']} graphs", flush=True)
