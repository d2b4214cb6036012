"""The C-ABI library loads and exports every symbol include/nrc/*.h declares; host-only entry
points behave; the C++ shim and the header compile. No GPU compute calls."""
import ctypes
import re
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
HEADERS = sorted((ROOT / "include" / "nrc").glob("*.h"))


def header_functions() -> list[str]:
    names = set()
    for h in HEADERS:
        text = re.sub(r"/\*.*?\*/", "", h.read_text(), flags=re.S)
        names |= set(re.findall(r"\b(nrc_[a-z0-9_]+)\s*\(", text))
    return sorted(names)


def test_header_declares_the_binding_list(nrc):
    assert header_functions() == sorted(nrc._lib.EXPORTS)


def test_library_exports_every_declared_symbol(nrc):
    syms = set(nrc._lib.exported_symbols())
    missing = [f for f in header_functions() if f not in syms]
    assert not missing, missing


def test_library_loads_and_host_entry_points(nrc):
    L = nrc._lib.lib()
    assert b"gfx950" in L.nrc_version()
    cfg = L.nrc_default_config(0)
    assert abs(cfg.learning_rate - 1e-3) < 1e-9 and abs(cfg.ema_decay - 0.99) < 1e-7
    assert abs(cfg.loss_scale - 128.0) < 1e-7 and abs(cfg.l2_reg - 1e-6) < 1e-12
    cfg_h = L.nrc_default_config(1)
    assert abs(cfg_h.learning_rate - 1e-2) < 1e-9 and abs(cfg_h.epsilon - 1e-15) < 1e-20
    h = ctypes.c_void_p()
    assert L.nrc_create(ctypes.byref(h)) == 0 and h.value
    # calls on a handle that was never init()ed fail cleanly, without touching the GPU
    assert L.nrc_infer(h, None, None, 0) == 3
    assert b"not initialised" in L.nrc_last_error()
    lr = ctypes.c_float()
    assert L.nrc_get_learning_rate(h, ctypes.byref(lr)) == 3
    assert L.nrc_set_config(h, 7) == 1  # std::invalid_argument("Unsupported input encoding")
    assert b"Unsupported input encoding" in L.nrc_last_error()
    assert L.nrc_set_config(h, 1) == 0 and L.nrc_last_error() == b""
    need = ctypes.c_size_t()
    assert L.nrc_get_config_json(h, None, 0, ctypes.byref(need)) == 0
    buf = ctypes.create_string_buffer(need.value)
    assert L.nrc_get_config_json(h, buf, need.value, None) == 0 and b"HashGrid" in buf.value
    assert L.nrc_set_config(h, 0) == 0 and L.nrc_last_error() == b""
    need = ctypes.c_size_t()
    assert L.nrc_get_config_json(h, None, 0, ctypes.byref(need)) == 0
    buf = ctypes.create_string_buffer(need.value)
    assert L.nrc_get_config_json(h, buf, need.value, None) == 0
    import json

    cfg_json = json.loads(buf.value.decode())
    assert cfg_json["network"] == {"activation": "ReLU", "n_hidden_layers": 5, "n_neurons": 64,
                                   "otype": "FullyFusedMLP", "output_activation": "ReLU"}
    assert [e["otype"] for e in cfg_json["encoding"]["nested"]] == ["TriangleWave", "OneBlob", "Identity"]
    assert cfg_json["loss"]["otype"] == "RelativeL2Luminance" and cfg_json["optimizer"]["otype"] == "EMA"
    assert L.nrc_destroy(h) == 0 and L.nrc_destroy(h) == 0  # idempotent
    assert L.nrc_infer(h, None, None, 16) == 2  # NRC_ERR_DESTROYED
    assert L.nrc_free(h) == 0
    assert L.nrc_create(None) == 1


def test_knob_values_are_range_checked(nrc):
    """nrc_debug_set_knob stored any integer, and train_shape >= 8 made the next training call divide by
    zero (SIGFPE). Out-of-range values are NRC_ERR_INVALID_ARGUMENT now and leave the knob unchanged (no GPU needed)."""
    L = nrc._lib
    bad = {"train_shape": [8, 100, -2], "train_kernel": [3, 31, 33, -5], "t16_groups": [0, 3], "hash_infer": [2, -2],
           "scatter_min": [0, 15, 1 << 21], "scatter_max": [7], "hash_feat_abl": [37, 127, 129], "dc_dw0_delay": [-2, 1 << 21],
           "hash_feat_p": [0, 12, 264], "peer_path": [5, -2], "px_polls": [0, -2, (1 << 21) + 1],
           "scatter_part": [17, -2], "scatter_compact": [17, -2], "hash_train_feat": [2, -2], "hash_adam": [1, -2],
           "train_fused": [2, -2], "fuse_mode": [5, -2], "tcnn_reentry": [2, -2], "train_prio": [3, -2]}
    for name, values in bad.items():
        before = L.get_knob(name)
        for v in values:
            with pytest.raises(nrc.NrcError) as e:
                L.set_knob(name, v)
            assert e.value.status == 1 and "out of range" in str(e.value), (name, v)
            assert L.get_knob(name) == before
    for name, v in [("train_shape", 7), ("train_kernel", 32), ("t16_groups", 1), ("scatter_min", 1024), ("peer_path", 0), ("peer_path", 4), ("px_polls", 1), ("scatter_part", 16), ("scatter_compact", 0), ("hash_train_feat", 1), ("hash_adam", 0), ("hash_feat_abl", 128), ("tcnn_reentry", 0), ("train_prio", 2)]:
        L.set_knob(name, v)
        assert L.get_knob(name) == v
        L.set_knob(name, -1)


def test_python_mirror_is_silent_after_destroy(nrc):
    net = nrc.Network()
    net.destroy()
    assert net.infer(1, 2, 16) is None and net.train(1, 2) is None  # reference: silent no-ops
    with pytest.raises(nrc.NrcError):
        net.getLearningRate()


def test_cpp_shim_compiles():
    src = ROOT / "tests" / "cpp" / "shim_compile.cpp"
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-std=c++17", "-fsyntax-only", f"-I{ROOT / 'include'}", str(src)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_layout_header_matches_python_constants(nrc):
    text = (ROOT / "include" / "nrc" / "layout.h").read_text()
    assert "#define NRC_NUM_PARAMS" in text
    assert nrc.NUM_PARAMS == 64 * 80 + 4 * 64 * 64 + 16 * 64 == 22528
    assert nrc.BATCH_SIZE == 65536 // 4


def test_frame_struct_layouts(nrc):
    """ctypes mirrors of include/nrc/frame.h structs have the C sizes (static_asserts in tests/cpp/shim_compile.cpp)."""
    F = nrc.frame
    assert ctypes.sizeof(F.NrcFrameBuffers) == 14 * 8
    assert ctypes.sizeof(F.NrcFrameParams) == 48
    assert F.TRAINING_RECORD_DTYPE.itemsize == 28 and F.END_VERTEX_DTYPE.itemsize == 16
