"""bench.py's power context of the roofline (CPU): the sampled window's mean socket power and clock, and the achieved
MFMA rate against the dense f16 peak scaled to that clock; no sampler (amdsmi missing) gives None, never an error."""
import bench


class FakeSampler:
    def __init__(self, w):
        self.w, self.stopped = w, False

    def window(self, t0, t1):
        return self.w

    def stop(self):
        self.stopped = True


def test_power_window_scales_the_peak_to_the_sampled_clock():
    s = FakeSampler({"samples": 30, "power_w": 1390.0, "gfx_mhz": 1800.0})
    r = bench.power_window(s, 0.0, 1.0, 1155.0)
    assert s.stopped
    assert r["socket_w"] == 1390.0 and r["gfx_mhz"] == 1800.0 and r["samples"] == 30
    assert abs(r["peak_at_clock_tflops"] - 2500.0 * 1800.0 / 2400.0) < 1e-9
    assert abs(r["frac_at_clock"] - 1155.0 / 1875.0) < 1e-12


def test_power_window_without_sampler_or_clock():
    assert bench.power_window(None, 0.0, 1.0, 1.0) is None
    r = bench.power_window(FakeSampler({"samples": 0}), 0.0, 1.0, 1.0)
    assert r == {"samples": 0, "socket_w": None, "gfx_mhz": None}
