"""ctypes binding of libnrc_amd.so (C-ABI: include/nrc/nrc_c.h).

The product path: there is no CPU fallback. If the HIP library is missing, importing the binding
raises, and every GPU entry point fails loudly.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
# NRC_LIB_PATH: alternate build of the same C-ABI -- libnrc_amd_debug.so (diagnostic stamps / clocks and the A/B
# kernels that lost their comparisons) or a build with other compile flags. The product path loads libnrc_amd.so.
PRODUCT_LIB_PATH = PKG_DIR / "libnrc_amd.so"
DEBUG_LIB_PATH = PKG_DIR / "libnrc_amd_debug.so"
LIB_PATH = Path(os.environ["NRC_LIB_PATH"]) if os.environ.get("NRC_LIB_PATH") else PRODUCT_LIB_PATH

NUM_PARAMS = 22528
GRAD_FLOATS = NUM_PARAMS + 4
HASH_NUM_PARAMS = 1012736
HASH_GRAD_FLOATS = HASH_NUM_PARAMS + 4
HASH_MLP_PARAMS = 21504                              # NRC_HASH_MLP_PARAMS
HASH_GRID_PARAMS = HASH_NUM_PARAMS - HASH_MLP_PARAMS  # NRC_HASH_GRID_PARAMS: int64 sums of nrc_train_grad_fixed
FIXED_MAX_RANKS = 63                                 # NRC_FIXED_MAX_RANKS
WIDE_NUM_PARAMS = 77824  # width-128 network (BASELINE configs[4])
PRECISION_F16, PRECISION_FP8, PRECISION_F16_ACC16 = 0, 1, 2  # nrc_precision (nrc_c.h)
BATCH_SIZE = 16384
# nrc_config.query_layout (layout.h): compact 15-float RadianceQuery, padded 16-float (USE_COMPACT_RADIANCE_QUERY 0)
QUERY_COMPACT, QUERY_PADDED = 0, 1
INPUT_DIMS = 15
OUTPUT_DIMS = 3

NRC_OK = 0
STATUS_NAMES = {
    0: "NRC_OK", 1: "NRC_ERR_INVALID_ARGUMENT", 2: "NRC_ERR_DESTROYED", 3: "NRC_ERR_NOT_INITIALIZED",
    4: "NRC_ERR_HIP", 5: "NRC_ERR_UNSUPPORTED", 6: "NRC_ERR_OUT_OF_MEMORY", 7: "NRC_ERR_INTERNAL",
}

# Every symbol include/nrc/*.h declares (checked by tests/test_abi.py).
EXPORTS = [
    "nrc_version", "nrc_last_error", "nrc_default_config", "nrc_create", "nrc_free", "nrc_init", "nrc_destroy",
    "nrc_train", "nrc_train_stream", "nrc_train_batch", "nrc_train_async", "nrc_infer", "nrc_infer_stream", "nrc_set_stream",
    "nrc_get_stream", "nrc_set_hyper_params", "nrc_set_config", "nrc_get_learning_rate", "nrc_get_config_json",
    "nrc_train_grad", "nrc_train_apply", "nrc_train_grad_fixed", "nrc_train_apply_fixed", "nrc_get_num_params", "nrc_get_grad_floats", "nrc_get_state", "nrc_set_state", "nrc_get_step",
    "nrc_set_step", "nrc_debug_encode_net",
    "nrc_comm_get_unique_id", "nrc_comm_init_rank", "nrc_comm_destroy", "nrc_set_comm", "nrc_get_comm_rank", "nrc_train_dp", "nrc_train_dp_async",
    "nrc_peer_exchange_handle", "nrc_peer_exchange_open", "nrc_peer_exchange_close", "nrc_peer_exchange_open_local",
    "nrc_encode", "nrc_debug_infer_variant", "nrc_debug_read_infer_clock", "nrc_debug_train_stamps", "nrc_debug_hash_scatter_inputs", "nrc_debug_infer_stamps", "nrc_debug_encode_fast",
    "nrc_debug_encode_fast_variant", "nrc_debug_infer_precision", "nrc_debug_fp8_convert", "nrc_debug_set_knob",
    "nrc_debug_get_knob", "nrc_debug_set_peer_seq",
    # include/nrc/frame.h (bound in frame.py)
    "nrc_accumulate_render_radiance", "nrc_infer_accumulate", "nrc_copy_radiance_to_output", "nrc_propagate_train_radiance",
    "nrc_accumulate_render_radiance_factored", "nrc_copy_radiance_to_output_factored", "nrc_propagate_train_radiance_factored",
    "nrc_accumulate_render_radiance_factored_padded", "nrc_copy_radiance_to_output_factored_padded",
    "nrc_propagate_train_radiance_factored_padded", "nrc_permute_train_data_padded",
    "nrc_generate_train_permutation", "nrc_sort_train_permutation_temp_bytes", "nrc_sort_train_permutation",
    "nrc_permute_train_data", "nrc_process_frame", "nrc_process_frame_shard",
    # include/nrc/stream.h (bound in stream.py)
    "nrc_stream_section_bytes", "nrc_stream_create", "nrc_stream_create_layout", "nrc_stream_query_layout",
    "nrc_stream_open", "nrc_stream_close",
    "nrc_stream_write_frame", "nrc_stream_next_frame", "nrc_stream_read_section",
]


class NrcConfig(ctypes.Structure):
    _fields_ = [("learning_rate", ctypes.c_float), ("beta1", ctypes.c_float), ("beta2", ctypes.c_float),
                ("epsilon", ctypes.c_float), ("l2_reg", ctypes.c_float), ("ema_decay", ctypes.c_float),
                ("loss_scale", ctypes.c_float), ("seed", ctypes.c_uint64), ("width", ctypes.c_uint32),
                ("infer_precision", ctypes.c_uint32), ("query_layout", ctypes.c_uint32)]


class NrcHyperParams(ctypes.Structure):
    _fields_ = [("learning_rate", ctypes.c_float)]


class NrcError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"{STATUS_NAMES.get(status, status)}: {msg}")
        self.status = status


_lib = None


def build() -> Path:
    subprocess.run(["make", "-s", "-C", str(PKG_DIR)], check=True)
    return LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise RuntimeError(f"HIP extension {LIB_PATH} is missing: run __graft_entry__.build() (no CPU fallback)")
    L = ctypes.CDLL(str(LIB_PATH))
    vp, fp, u32 = ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32
    st = ctypes.c_int
    sigs = {
        "nrc_version": (ctypes.c_char_p, []),
        "nrc_last_error": (ctypes.c_char_p, []),
        "nrc_default_config": (NrcConfig, [ctypes.c_int]),
        "nrc_create": (st, [ctypes.POINTER(vp)]),
        "nrc_free": (st, [vp]),
        "nrc_init": (st, [vp, vp, ctypes.c_int, ctypes.POINTER(NrcConfig), ctypes.c_int]),
        "nrc_destroy": (st, [vp]),
        "nrc_train": (st, [vp, fp, fp, ctypes.POINTER(ctypes.c_float)]),
        "nrc_train_stream": (st, [vp, fp, fp, vp, ctypes.POINTER(ctypes.c_float)]),
        "nrc_train_batch": (st, [vp, fp, fp, u32, ctypes.POINTER(ctypes.c_float)]),
        "nrc_train_async": (st, [vp, fp, fp, u32, fp]),
        "nrc_infer": (st, [vp, fp, fp, u32]),
        "nrc_infer_stream": (st, [vp, fp, fp, u32, vp]),
        "nrc_set_stream": (st, [vp, vp]),
        "nrc_get_stream": (st, [vp, ctypes.POINTER(vp)]),
        "nrc_set_hyper_params": (st, [vp, ctypes.POINTER(NrcHyperParams)]),
        "nrc_set_config": (st, [vp, ctypes.c_int]),
        "nrc_get_learning_rate": (st, [vp, ctypes.POINTER(ctypes.c_float)]),
        "nrc_get_config_json": (st, [vp, ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]),
        "nrc_train_grad": (st, [vp, fp, fp, u32, u32, fp]),
        "nrc_train_apply": (st, [vp, fp, ctypes.POINTER(ctypes.c_float)]),
        "nrc_train_grad_fixed": (st, [vp, fp, fp, u32, u32, fp, vp]),
        "nrc_train_apply_fixed": (st, [vp, fp, vp, ctypes.POINTER(ctypes.c_float)]),
        "nrc_get_state": (st, [vp, ctypes.c_int, fp]),
        "nrc_set_state": (st, [vp, ctypes.c_int, fp]),
        "nrc_get_step": (st, [vp, ctypes.POINTER(u32)]),
        "nrc_get_num_params": (st, [vp, ctypes.POINTER(ctypes.c_uint64)]),
        "nrc_get_grad_floats": (st, [vp, ctypes.POINTER(ctypes.c_uint64)]),
        "nrc_debug_encode_net": (st, [vp, fp, fp, u32, vp]),
        "nrc_set_step": (st, [vp, u32]),
        "nrc_comm_get_unique_id": (st, [vp]),
        "nrc_comm_init_rank": (st, [ctypes.POINTER(vp), vp, ctypes.c_int, ctypes.c_int]),
        "nrc_comm_destroy": (st, [vp]),
        "nrc_set_comm": (st, [vp, vp]),
        "nrc_get_comm_rank": (st, [vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
        "nrc_train_dp": (st, [vp, fp, fp, u32, u32, ctypes.POINTER(ctypes.c_float)]),
        "nrc_train_dp_async": (st, [vp, fp, fp, u32, u32, fp]),
        "nrc_peer_exchange_handle": (st, [vp, ctypes.c_int, vp]),
        "nrc_peer_exchange_open": (st, [vp, ctypes.c_int, ctypes.c_int, vp]),
        "nrc_peer_exchange_close": (st, [vp]),
        "nrc_peer_exchange_open_local": (st, [ctypes.POINTER(vp), ctypes.c_int]),
        "nrc_debug_set_peer_seq": (st, [vp, u32]),
        "nrc_encode": (st, [fp, fp, u32, vp]),
        "nrc_debug_infer_variant": (st, [vp, ctypes.c_int, fp, fp, u32, vp]),
        "nrc_debug_read_infer_clock": (st, [vp, u32, ctypes.POINTER(u32)]),
        "nrc_debug_train_stamps": (st, [vp, fp, fp, u32, vp]),
        "nrc_debug_hash_scatter_inputs": (st, [vp, vp, vp, u32]),
        "nrc_debug_infer_stamps": (st, [vp, fp, fp, u32, vp, ctypes.POINTER(ctypes.c_uint64)]),
        "nrc_debug_encode_fast": (st, [fp, fp, u32, vp]),
        "nrc_debug_encode_fast_variant": (st, [ctypes.c_int, fp, fp, u32, vp]),
        "nrc_debug_infer_precision": (st, [vp, ctypes.c_int, fp, fp, u32, vp]),
        "nrc_debug_fp8_convert": (st, [fp, fp, u32, ctypes.c_int, vp]),
        "nrc_debug_set_knob": (st, [ctypes.c_char_p, ctypes.c_int]),
        "nrc_debug_get_knob": (st, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]),
    }
    for name, (res, args) in sigs.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def check(status: int) -> None:
    if status != NRC_OK:
        raise NrcError(status, lib().nrc_last_error().decode(errors="replace"))


def set_knob(name: str, value: int) -> None:
    """Process-wide A/B knob of the library (nrc_debug_set_knob; -1 = the production choice)."""
    check(lib().nrc_debug_set_knob(name.encode(), int(value)))


def get_knob(name: str) -> int:
    v = ctypes.c_int()
    check(lib().nrc_debug_get_knob(name.encode(), ctypes.byref(v)))
    return v.value


def is_debug_library() -> bool:
    return LIB_PATH.resolve() == DEBUG_LIB_PATH.resolve()


def last_error() -> str:
    return lib().nrc_last_error().decode(errors="replace")


def exported_symbols() -> list[str]:
    """Dynamic symbols exported by the library (via the ELF .dynsym, no GPU needed)."""
    out = subprocess.run(["nm", "-D", "--defined-only", str(LIB_PATH)], check=True, capture_output=True, text=True)
    return sorted({line.split()[-1] for line in out.stdout.splitlines() if line.strip()})


def default_env_ok() -> bool:
    return os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0") == "0"
