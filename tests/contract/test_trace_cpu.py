"""DeviceStages bookkeeping with fake events on a CPU box."""
from agent_tpu_amd.utils.trace import DeviceStages


class FakeEvent:
    def __init__(self, t):
        self.t = t

    def elapsed_time(self, other):
        return other.t - self.t


def test_device_stages_sum_span_overlap():
    d = DeviceStages()
    E = FakeEvent
    # slot 0: h2d 0-1, tokenize 1-2, encoder 2-10; slot 1 (other stream) encoder 6-14
    d.add("h2d", E(0.0), E(1.0))
    d.add("tokenize", E(1.0), E(2.0))
    d.add("encoder", E(2.0), E(10.0))
    d.add("encoder", E(6.0), E(14.0))
    out = d.resolve({"host_drain_ms": 3.0})
    assert out["device_h2d_ms"] == 1.0 and out["device_tokenize_ms"] == 1.0
    assert out["device_encoder_ms"] == 16.0
    assert out["device_span_ms"] == 14.0
    assert out["device_overlap"] == round(18.0 / 14.0, 3)
    assert out["host_drain_ms"] == 3.0
    assert d.pairs == [] and d.resolve({}) == {}
