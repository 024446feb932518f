"""worker_sizing: CPU formulas (reference worker_sizing.py:44-124 goldens),
AMD GPU discovery from a fake KFD topology, visibility filters, HBM-derived
batch sizing, TPU schema stability."""
import os
import types

import pytest

import worker_sizing as ws

GIB = 1 << 30


def _node(root, idx, props, banks=()):
    d = os.path.join(root, str(idx))
    os.makedirs(os.path.join(d, "mem_banks"))
    with open(os.path.join(d, "properties"), "w") as f:
        for k, v in props.items():
            f.write(f"{k} {v}\n")
    for b, (heap, size) in enumerate(banks):
        bd = os.path.join(d, "mem_banks", str(b))
        os.makedirs(bd)
        with open(os.path.join(bd, "properties"), "w") as f:
            f.write(f"heap_type {heap}\nsize_in_bytes {size}\n")


@pytest.fixture
def kfd(tmp_path, monkeypatch):
    root = str(tmp_path / "nodes")
    _node(root, 0, {"simd_count": 0, "cpu_cores_count": 64}, [(0, 512 * GIB)])
    for i in (1, 2):
        _node(root, i, {"simd_count": 1024, "simd_per_cu": 4, "gfx_target_version": 90500},
              [(1, 288 * GIB), (0, 64 * GIB)])
    monkeypatch.setenv("ATPU_KFD_TOPOLOGY", root)
    for v in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "GPU_DISABLED",
              "CLASSIFY_BATCH_ROWS", "DP_WORLD_SIZE", "GPU_ONLY", "TPU_ONLY"):
        monkeypatch.delenv(v, raising=False)
    return root


def test_kfd_discovery(kfd):
    g = ws.detect_gpu()
    assert g["gpu_present"] and g["gpu_count"] == 2 and g["vendor"] == "amd"
    assert g["vram_gb"] == 288.0 and g["hbm_gb"] == [288.0, 288.0]
    d = g["devices"][0]
    assert d == {"index": 0, "name": "gfx950", "arch": "gfx950", "total_memory_bytes": 288 * GIB,
                 "compute_units": 256}
    assert g["max_gpu_workers"] == 2 and g["dp_world_size"] == 2
    assert g["classify_batch_rows"] == 1024  # capped: GEMMs saturate near 128k tokens


@pytest.mark.parametrize("var", ["HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"])
def test_visibility_filters(kfd, monkeypatch, var):
    monkeypatch.setenv(var, "1")
    g = ws.detect_gpu()
    assert g["gpu_count"] == 1 and g["devices"][0]["index"] == 0
    for hidden in ("none", "-1", ""):
        monkeypatch.setenv(var, hidden)
        assert ws.detect_gpu()["gpu_present"] is False


def test_gpu_disabled_and_batch_override(kfd, monkeypatch):
    monkeypatch.setenv("CLASSIFY_BATCH_ROWS", "333")
    monkeypatch.setenv("DP_WORLD_SIZE", "1")
    g = ws.detect_gpu()
    assert g["classify_batch_rows"] == 333 and g["dp_world_size"] == 1
    monkeypatch.setenv("GPU_DISABLED", "yes")
    assert ws.detect_gpu() == {"gpu_present": False, "gpu_count": 0, "vram_gb": None, "devices": [],
                               "max_gpu_workers": 0}


def test_batch_rows_from_small_hbm(monkeypatch):
    for v in ("CLASSIFY_BATCH_ROWS", "CLASSIFY_SEQ_LEN", "HBM_RESERVE_GB", "MODEL_LRU_GB", "CLASSIFY_BATCH_ROWS_CAP"):
        monkeypatch.delenv(v, raising=False)
    assert ws.classify_batch_rows(288 * GIB) == 1024
    # 12 GiB: 8 reserved, 3 for the model LRU -> 1 GiB of activations / 3.16 MB per row -> 339 -> 320
    assert ws.classify_batch_rows(12 * GIB) == 320
    assert ws.classify_batch_rows(10 * GIB) == 1  # nothing left after reserve + LRU: one row at a time


def _presets():
    from agent_tpu_amd.models import bart, bert, t5

    return bert, t5, bart


def test_sizing_tables_match_model_presets():
    """worker_sizing stays torch-free with its own shape tables; they must match the models."""
    bert, t5, bart = _presets()
    for name, (H, I, L, V, P) in ws.CLASSIFY_DIMS.items():
        c = bert.config_for(name)
        assert (c.hidden, c.intermediate, c.layers, c.vocab_size, c.max_positions) == (H, I, L, V, P), name
    for name, dims in ws.SUMMARIZE_DIMS.items():
        c = (t5 if name.startswith("t5") else bart).config_for(name)
        assert (c.d_model, c.d_ff, c.enc_layers, c.dec_layers, c.vocab_size) == dims, name
    from agent_tpu_amd.tokenizer import DEFAULT_MAX_ROW_BYTES

    assert ws.CLASSIFY_MAX_ROW_BYTES == DEFAULT_MAX_ROW_BYTES


def test_model_aware_capacity_288gb(kfd, monkeypatch):
    """per-model numbers a 288 GB MI355X advertises, and the engines use them."""
    for v in ("CLASSIFY_SEQ_LEN", "HBM_RESERVE_GB", "MODEL_LRU_GB", "SUMMARIZE_BATCH_DOCS", "RISK_CHUNK_ROWS",
              "RISK_STAGING_MB", "GPU_MODEL_PATH", "CLASSIFY_MODEL", "CLASSIFY_BATCH_ROWS_CAP"):
        monkeypatch.delenv(v, raising=False)
    cap = ws.detect_gpu()["capacity"]
    # per-row bytes: slots x (text staging + ids + S*2*(6H + I) activations + LN statistics)
    assert ws.classify_row_bytes("bert-base", 128) == 3_161_104
    assert ws.classify_row_bytes("bert-large", 128) == 4_209_680
    assert cap["classify_batch_rows"] == {"bert-base": 1024, "bert-large": 1024}  # token target binds at 288 GB
    assert cap["classify_seq_len"] == 128
    # per-document bytes of a beam search at the reference's settings (src 1024, 4 beams, max 130)
    assert ws.summarize_doc_bytes("t5-base") == 72_822_144
    assert ws.summarize_doc_bytes("bart-large-cnn") == 97_127_232
    assert cap["summarize_batch_docs"] == {"t5-base": 1024, "bart-large-cnn": 1024}
    assert cap["risk_chunk_rows"] == (256 << 20) // 56  # 256 MiB of pinned staging / (2 slots x (24 + 4) B)
    # sequence length moves the token target; HBM binds on a small device
    monkeypatch.setenv("CLASSIFY_SEQ_LEN", "512")
    assert ws.detect_gpu()["capacity"]["classify_batch_rows"]["bert-large"] == 256
    assert ws.classify_batch_rows(12 * GIB, "bert-large", 128) == 192  # 1 GiB / 5.26 MB = 204 -> 192
    assert ws.summarize_batch_docs(24 * GIB, "bart-large-cnn") == 110  # 10 GiB / 97.1 MB
    # the served classify model's number is the top-level one
    monkeypatch.setenv("GPU_MODEL_PATH", "bert-large?labels=4")
    assert ws.detect_gpu()["classify_batch_rows"] == 256


def test_engines_use_the_advertised_sizes(monkeypatch):
    """The engine batch equals the advertised one (CPU: the runtime assumes a 288 GB device)."""
    for v in ("CLASSIFY_BATCH_ROWS", "CLASSIFY_SEQ_LEN", "HBM_RESERVE_GB", "MODEL_LRU_GB", "SUMMARIZE_BATCH_DOCS"):
        monkeypatch.delenv(v, raising=False)
    from ops._gpu_runtime import _auto_batch_rows

    for m, seq in (("bert-base", 128), ("bert-large", 128), ("bert-large", 512), ("bert-base", 64)):
        assert _auto_batch_rows(m, seq) == ws.classify_batch_rows(288 * GIB, m, seq)
    assert _auto_batch_rows("bert-base", 64) == 2048
    import torch

    from agent_tpu_amd.runtime.summarize import SummarizeEngine, build_model

    model, _ = build_model("t5-tiny", device=torch.device("cpu"), seed=0, fp32=True)
    eng = SummarizeEngine(model, 1024)
    c = model.cfg
    assert eng.max_batch_docs == ws.summarize_batch_docs(288 * GIB, (c.d_model, c.d_ff, c.enc_layers,
                                                                     c.dec_layers, c.vocab_size), 1024)
    assert SummarizeEngine(model, 64, max_batch_docs=2).max_batch_docs == 2


def test_cpu_formulas_match_reference_probe(monkeypatch):
    fake = types.SimpleNamespace(cpu_count=lambda logical=True: 8,
                                 virtual_memory=lambda: types.SimpleNamespace(available=64 * GIB))
    monkeypatch.setattr(ws, "psutil", fake)
    for v in ("CPU_RESERVED_CORES_FLOOR", "CPU_RESERVED_CORES_CAP", "CPU_PIPELINE_FACTOR", "CPU_MIN_WORKERS",
              "CPU_SOFT_CAP_MULTIPLIER", "CPU_PER_WORKER_BYTES"):
        monkeypatch.delenv(v, raising=False)
    c = ws.detect_cpu()
    # [probe] in SURVEY.md §2.1 #30: 8 cores -> reserved 2, usable 6, target 24, cap 48
    assert (c["total_cores"], c["reserved_cores"], c["usable_cores"]) == (8, 2, 6)
    assert c["target_inflight_workers"] == 24 and c["cpu_soft_cap_workers"] == 48 == c["max_cpu_workers"]
    monkeypatch.setenv("CPU_PER_WORKER_BYTES", str(8 * GIB))
    assert ws.detect_cpu()["cpu_soft_cap_workers"] == 8  # RAM cap
    monkeypatch.setenv("CPU_PIPELINE_FACTOR", "not-a-number")
    assert ws.detect_cpu()["pipeline_factor"] == 4.0  # parse errors fall back to defaults


def test_profile_schema_and_only_modes(kfd, monkeypatch):
    p = ws.build_worker_profile()
    assert set(p) == {"cpu", "gpu", "tpu", "workers"}
    assert p["tpu"] == {"tpu_present": False, "tpu_kind": None, "devices": [], "max_tpu_workers": 0}
    assert p["workers"]["max_total_workers"] == p["cpu"]["cpu_soft_cap_workers"] + 2
    monkeypatch.setenv("GPU_ONLY", "1")
    p = ws.build_worker_profile()
    assert p["cpu"]["max_cpu_workers"] == 1 and p["workers"]["max_total_workers"] == 3
    monkeypatch.setenv("TPU_NAME", "x")
    assert ws.detect_tpu()["tpu_kind"] == "hinted" and ws.detect_tpu()["tpu_present"] is False
    monkeypatch.setenv("TPU_DISABLED", "on")
    assert ws.detect_tpu()["tpu_kind"] is None


@pytest.mark.parametrize("raw,val", [("1", True), ("TRUE", True), ("y", True), ("on", True), ("0", False),
                                     ("no", False), ("off", False), ("maybe", None), (None, None)])
def test_env_bool(monkeypatch, raw, val):
    if raw is None:
        monkeypatch.delenv("X_BOOL", raising=False)
    else:
        monkeypatch.setenv("X_BOOL", raw)
    assert ws.env_bool("X_BOOL", None) is val


def test_gpu_busy_from_fake_drm(tmp_path, monkeypatch):
    """gpu_util[]: amdgpu cards only (vendor 0x1002), card order, connectors skipped."""
    def card(name, vendor, busy=None):
        d = tmp_path / name / "device"
        d.mkdir(parents=True)
        (d / "vendor").write_text(vendor + "\n")
        if busy is not None:
            (d / "gpu_busy_percent").write_text(f"{busy}\n")

    card("card1", "0x1002", 37)
    card("card10", "0x1002", 100)
    card("card2", "0x1002", 0)
    card("card3", "0x8086", 50)  # not AMD
    (tmp_path / "card1-DP-1").mkdir()  # connector
    (tmp_path / "renderD128").mkdir()
    monkeypatch.setenv("ATPU_DRM_ROOT", str(tmp_path))
    assert ws.probe_gpu_busy() == [0.37, 0.0, 1.0]
    import app

    assert app.gpu_metrics()["gpu_util"] == [0.37, 0.0, 1.0]
    monkeypatch.setenv("ATPU_DRM_ROOT", str(tmp_path / "missing"))
    assert ws.probe_gpu_busy() == []
