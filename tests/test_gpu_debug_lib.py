"""The product / debug library split (VERDICT r02 housekeeping).

libnrc_amd.so (the product, what every other test and bench.py load) holds the production kernels only; the
diagnostic builds (phase stamps, in-kernel clocks) and the A/B kernels that lost their comparisons (inference variants
0/23/30/40, the 16x16x32 inference kernel 50/51, the width-128 1024-thread variant, the 4-wave t16 training kernel)
live in libnrc_amd_debug.so, built from the same sources with NRC_DEBUG_KERNELS=1 and loaded by tools through
NRC_LIB_PATH. Here: the product library refuses the debug entry points with NRC_ERR_UNSUPPORTED, and ONE subprocess
re-runs the A/B variant parity tests and the stamp entry points against the debug library.
"""
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def test_debug_entry_points(nrc, dev):
    import torch

    lib = nrc._lib.lib()
    net = nrc.Network()
    net.init(stream=torch.cuda.current_stream())
    b = 2048
    q, t = nrc.synthetic.cornell_batch(b, seed=5)
    q, t = torch.from_numpy(q).to(dev), torch.from_numpy(t).to(dev)
    out = torch.zeros((4096, 3), device=dev)
    stamps = torch.zeros(64 * 16 * 8, dtype=torch.int64, device=dev)
    calls = {
        "train_stamps": lambda: lib.nrc_debug_train_stamps(net._h, q.data_ptr(), t.data_ptr(), b, stamps.data_ptr()),
        "variant_23": lambda: lib.nrc_debug_infer_variant(net._h, 23, q.data_ptr(), out.data_ptr(), 2048, None),
        "variant_50": lambda: lib.nrc_debug_infer_variant(net._h, 50, q.data_ptr(), out.data_ptr(), 2048, None),
    }
    try:
        for name, call in calls.items():
            st = call()
            torch.cuda.synchronize()
            if nrc._lib.is_debug_library():
                assert st == 0, (name, nrc._lib.last_error())
            else:
                assert st == 5, (name, st)  # NRC_ERR_UNSUPPORTED
                assert "debug library" in nrc._lib.last_error()
        if nrc._lib.is_debug_library():
            s = stamps.cpu().numpy()[:64 * 6 * 16].reshape(64, 6, 16)  # dc shape 7: 64 blocks x 6 waves
            assert (np.diff(s[:, 0, :14], axis=1) >= 0).all(), "chain-wave stamps must be monotone"
        # variant 47 (the product kernel) is available in both
        nrc._lib.check(lib.nrc_debug_infer_variant(net._h, 47, q.data_ptr(), out.data_ptr(), 2048, None))
    finally:
        net.destroy()


@pytest.mark.skipif(os.environ.get("NRC_LIB_PATH") is not None, reason="already running under an alternate library")
def test_debug_library_variants_in_subprocess():
    dbg = ROOT / "neural-radiance-caching_amd" / "libnrc_amd_debug.so"
    assert dbg.exists(), "libnrc_amd_debug.so is built by __graft_entry__.build() / make"
    env = dict(os.environ, NRC_LIB_PATH=str(dbg))
    cmd = [sys.executable, "-u", "-m", "pytest", "-x", "-q", "-m", "gpu", "-p", "no:cacheprovider",
           "--timeout", "120", "--timeout-method", "thread",
           "tests/test_gpu_parity.py::test_every_infer_variant_per_sample",
           "tests/test_gpu_parity.py::test_early_first_tile_variants_bitwise",
           "tests/test_gpu_train_dc.py::test_t16_64_sample_blocks",
           "tests/test_gpu_parity.py::test_pooled_variant_bitwise_and_reusable",
           "tests/test_gpu_wide.py::test_wide_kernel_variant_bit_identical",
           "tests/test_gpu_wide.py::test_wide_fp8_byte_relu_variant_bit_identical",
           "tests/test_gpu_debug_lib.py::test_debug_entry_points",
           "tests/test_gpu_train_dc.py::test_dc_gradient_is_deterministic_with_a_slow_dw_wave",
           "tests/test_gpu_train_dc.py::test_dc_protocol_timeout_is_reported"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    print(r.stdout[-3000:])
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    tail = r.stdout.strip().splitlines()[-1]
    assert " passed" in tail and "skipped" not in tail, tail  # every A/B variant ran under the debug library
