"""Registry semantics (ref /root/reference/ops/__init__.py)."""
import pytest

import ops
import ops_loader


@pytest.fixture(autouse=True)
def _clean_tasks(monkeypatch):
    monkeypatch.delenv("TASKS", raising=False)
    ops._reset_for_tests()
    yield
    ops._reset_for_tests()


def test_unset_all_star_enable_default_ops(monkeypatch):
    base = ops.list_ops()
    assert base == sorted(n for n in ops.OP_TO_MODULE if n not in ops.OPT_IN_OPS)
    for kw in ("*", "all", "ALL", " all , "):
        monkeypatch.setenv("TASKS", kw)
        assert ops.list_ops() == base


def test_none_and_exact_names_case_sensitive(monkeypatch):
    monkeypatch.setenv("TASKS", "none")
    assert ops.list_ops() == []
    monkeypatch.setenv("TASKS", "echo,csv_shard")
    assert ops.list_ops() == ["csv_shard", "echo"]
    monkeypatch.setenv("TASKS", "ECHO")
    assert ops.list_ops() == []


def test_get_op_error_messages(monkeypatch):
    with pytest.raises(ValueError, match=r"Unknown op 'nonexistent'\. Allowed ops: \["):
        ops.get_op("nonexistent")
    monkeypatch.setenv("TASKS", "echo")
    with pytest.raises(ValueError, match=r"Op 'map_tokenize' is not enabled by TASKS\. Enabled ops: \['echo'\]"):
        ops.get_op("map_tokenize")


def test_failed_import_reported_once(monkeypatch, capsys):
    monkeypatch.setitem(ops.OP_TO_MODULE, "ghost", "ghost_module_does_not_exist")
    for _ in range(3):
        with pytest.raises(ValueError, match=r"Unknown or failed op 'ghost'.*Also saw op import errors: "
                                             r"ghost_module_does_not_exist => ModuleNotFoundError"):
            ops.get_op("ghost")
    assert len(ops.OPS_LOAD_ERRORS) == 1  # the reference appended on every call
    assert capsys.readouterr().out.count("[ops] ERROR: failed to import ops.ghost_module_does_not_exist") == 1


def test_aliases_resolve_to_same_handler():
    assert ops.get_op("csv_shard") is ops.get_op("read_csv_shard")
    assert ops.get_op("map_classify_tpu").__name__ == "map_classify_tpu"
    assert ops.get_op("map_classify").__name__ == "map_classify"


def test_opt_in_triggers(monkeypatch):
    assert "trigger_oracle" not in ops.list_ops()
    with pytest.raises(ValueError, match="not enabled"):
        ops.get_op("trigger_sap")
    monkeypatch.setenv("TASKS", "all,trigger_sap")
    assert "trigger_sap" in ops.list_ops() and "trigger_oracle" not in ops.list_ops()
    assert callable(ops.get_op("trigger_sap"))


def test_every_mapped_module_exists():
    import importlib.util

    for name, mod in ops.OP_TO_MODULE.items():
        assert importlib.util.find_spec(f"ops.{mod}") is not None, name


def test_ops_loader(monkeypatch):
    got = ops_loader.load_ops(["echo", "map_tokenize"])
    assert set(got) == {"echo", "map_tokenize"}
    with pytest.raises(ValueError):
        ops_loader.load_ops(["echo", "nope"])
    ok, bad = ops_loader.load_ops_lenient(["echo", "nope"])
    assert list(ok) == ["echo"] and bad[0][0] == "nope"


def test_every_op_has_a_contract():
    """Reference contract format (ops/map_classify_tpu.CONTRACT.md:1-26): title + 4 sections."""
    import os

    here = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "ops")
    modules = set(ops.OP_TO_MODULE.values())
    for mod in modules:
        path = os.path.join(here, f"{mod}.CONTRACT.md")
        assert os.path.exists(path), f"missing {path}"
        text = open(path).read()
        assert text.startswith("# ") and "— Contract (v0)" in text.splitlines()[0], path
        for sec in ("## Purpose", "## Inputs (payload)", "## Outputs", "## Notes"):
            assert sec in text, (path, sec)


def test_device_fault_marks_the_faulting_ranks_device(monkeypatch):
    """DP errors name global ranks ("rank K: ..."; rank K drives device K): a
    HIP fault on rank 2 marks device 2, an ordinary error on rank 1 marks
    nothing, and an un-prefixed fault marks this process's own device."""
    import types

    import app
    from agent_tpu_amd.runtime import health

    monkeypatch.setattr(health, "_unhealthy", {})
    monkeypatch.setattr(health, "_last", {"ok": True, "devices": [], "healthy": [0, 1, 2, 3], "unhealthy": {}})
    monkeypatch.setattr(app, "worker_profile", lambda h, caps=None: {"health": h})
    me = types.SimpleNamespace(health=health.last(), profile=None, caps=["map_classify"])
    app.Agent._note_device_fault(me, "rank 1: ValueError: bad; rank 2: RuntimeError: hipErrorLaunchFailure: boom")
    assert sorted(health._unhealthy) == [2] and health.last()["healthy"] == [0, 1, 3]
    assert me.profile == {"health": health.last()}
    monkeypatch.setenv("LOCAL_RANK", "3")
    app.Agent._note_device_fault(me, "RuntimeError: HIP error: illegal memory access")
    assert sorted(health._unhealthy) == [2, 3]
    app.Agent._note_device_fault(me, "ValueError: payload.values must be a list")
    assert sorted(health._unhealthy) == [2, 3]
