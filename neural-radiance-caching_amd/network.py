"""Host-side mirror of the reference's ``nrc::Network`` (/root/reference/nrc/inc/NRCNetwork.h:20-75)
over the C-ABI (include/nrc/nrc_c.h).

Method names, argument meaning and error behaviour follow the reference:

=====================================  =========================================================
reference (NRCNetwork.h)               here
=====================================  =========================================================
``Network()`` / ``~Network()``         ``Network()`` / garbage collection (``nrc_create``/``nrc_free``)
``init<Verbose>(stream, encoding)``    ``init(stream, encoding, verbose=False)``
``destroy()``                          ``destroy()``
``train(in, tgt, loss_h)``             ``train(inputs, targets, loss=False)`` -> loss or None
``train(in, tgt, stream, loss_h)``     ``train(inputs, targets, stream=s, loss=...)``
``infer(in, out, n)``                  ``infer(inputs, outputs, num_inputs)``
``infer(in, out, n, stream)``          ``infer(inputs, outputs, num_inputs, stream=s)``
``setStream`` / ``setHyperParams``     ``setStream`` / ``setHyperParams`` (+ snake_case aliases)
``setConfig`` / ``getLearningRate``    ``setConfig`` / ``getLearningRate``
=====================================  =========================================================

As in the reference (NRCNetwork.cu:43, :66), ``train`` / ``infer`` after ``destroy()`` are silent
no-ops; the C-ABI reports them as ``NRC_ERR_DESTROYED``. Buffers are device pointers: a CUDA
(HIP) ``torch.Tensor`` (float32, contiguous) or a raw integer address. ``train`` consumes exactly
``BATCH_SIZE`` = 16384 samples (NRCNetwork.cu:51-52).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from enum import IntEnum

import numpy as np

from . import _lib
from ._lib import (BATCH_SIZE, GRAD_FLOATS, HASH_GRID_PARAMS, NUM_PARAMS, QUERY_PADDED, NrcConfig, NrcError,
                   NrcHyperParams, check, lib)

NRC_ERR_DESTROYED = 2


class InputEncoding(IntEnum):
    """nrc::InputEncoding (neural_radiance_caching.h:24-27), plus the FrequencySH extension (layout.h)."""
    Frequency = 0
    Hash = 1
    FrequencySH = 2


class StateSlot(IntEnum):
    PARAMS = 0
    INFER = 1
    EMA = 2
    ADAM_M = 3
    ADAM_V = 4


@dataclass
class HyperParams:
    """nrc::HyperParams (NRCNetwork.h:10-13)."""
    learningRate: float


_DTYPE_OK: dict = {}  # dtype objects already checked against each dtype name


def _dev_ptr(x, what: str, min_elems: int | None = None, dtype: str = "torch.float32") -> int:
    if x is None:
        raise ValueError(f"{what}: null buffer")
    if isinstance(x, int):
        return x
    # torch.Tensor (duck-typed so that importing this module does not require torch)
    if hasattr(x, "data_ptr"):
        if not x.is_cuda:
            raise ValueError(f"{what}: tensor must live on the GPU")
        dt = x.dtype
        if dt not in _DTYPE_OK.get(dtype, ()):  # the string compare only once per dtype (a hot-path call)
            if str(dt) != dtype:
                raise ValueError(f"{what}: tensor must be {dtype.split('.')[-1]}")
            _DTYPE_OK.setdefault(dtype, set()).add(dt)
        if not x.is_contiguous():
            raise ValueError(f"{what}: tensor must be contiguous")
        if min_elems is not None and x.numel() < min_elems:
            raise ValueError(f"{what}: needs at least {min_elems} elements, got {x.numel()}")
        return int(x.data_ptr())
    raise TypeError(f"{what}: expected a CUDA tensor or an integer device address, got {type(x)}")


def _stream_ptr(stream) -> int | None:
    if stream is None:
        return None
    if isinstance(stream, int):
        return stream
    if hasattr(stream, "cuda_stream"):
        return int(stream.cuda_stream)
    raise TypeError(f"stream: expected torch.cuda.Stream or int, got {type(stream)}")


def current_stream() -> int:
    import torch
    return int(torch.cuda.current_stream().cuda_stream)


class Network:
    """MI355X-native drop-in for nrc::Network."""

    def __init__(self):
        h = ctypes.c_void_p()
        check(lib().nrc_create(ctypes.byref(h)))
        self._h = h
        self._lib = lib()
        self.query_dims = 15

    # ---- lifecycle ---------------------------------------------------------------------------
    def init(self, stream=None, encoding: InputEncoding = InputEncoding.Frequency, verbose: bool = False,
             config: NrcConfig | None = None) -> None:
        s = _stream_ptr(stream)
        cfg = ctypes.byref(config) if config is not None else None
        check(self._lib.nrc_init(self._h, s, int(encoding), cfg, int(bool(verbose))))
        self.encoding = InputEncoding(int(encoding))
        # floats per RadianceQuery record (nrc_config.query_layout: compact 15, padded 16)
        self.query_dims = 16 if config is not None and int(config.query_layout) == QUERY_PADDED else 15

    def destroy(self) -> None:
        check(self._lib.nrc_destroy(self._h))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                self._lib.nrc_free(h)
                self._h = ctypes.c_void_p()
            except Exception:  # interpreter shutdown: module globals may already be gone
                pass

    # ---- hot path ----------------------------------------------------------------------------
    def train(self, inputs, targets, stream=None, loss: bool = False):
        """One training step on BATCH_SIZE samples; returns the batch loss if loss=True (blocking)."""
        pi = _dev_ptr(inputs, "inputs", BATCH_SIZE * self.query_dims if hasattr(inputs, "numel") else None)
        pt = _dev_ptr(targets, "targets", BATCH_SIZE * 3 if hasattr(targets, "numel") else None)
        lh = ctypes.c_float(float("nan"))
        lp = ctypes.byref(lh) if loss else None
        if stream is None:
            st = self._lib.nrc_train(self._h, pi, pt, lp)
        else:
            st = self._lib.nrc_train_stream(self._h, pi, pt, _stream_ptr(stream), lp)
        if st == NRC_ERR_DESTROYED:
            return None
        check(st)
        return lh.value if loss else None

    def infer(self, inputs, outputs, numInputs: int, stream=None) -> None:
        n = int(numInputs)
        if n < 0 or n > 0xFFFFFFFF:
            raise ValueError("numInputs out of range")
        pi = _dev_ptr(inputs, "inputs", n * self.query_dims if hasattr(inputs, "numel") else None)
        po = _dev_ptr(outputs, "outputs", n * 3 if hasattr(outputs, "numel") else None)
        if stream is None:
            st = self._lib.nrc_infer(self._h, pi, po, n)
        else:
            st = self._lib.nrc_infer_stream(self._h, pi, po, n, _stream_ptr(stream))
        if st == NRC_ERR_DESTROYED:
            return None
        check(st)

    def infer_precision(self, precision: int, inputs, outputs, numInputs: int, stream=None) -> None:
        """Width-128 network: inference through the f16 (0) or FP8 (1) weight image, whatever infer_precision the
        handle was configured with (A/B timing, parity tests)."""
        n = int(numInputs)
        pi = _dev_ptr(inputs, "inputs", n * self.query_dims if hasattr(inputs, "numel") else None)
        po = _dev_ptr(outputs, "outputs", n * 3 if hasattr(outputs, "numel") else None)
        check(self._lib.nrc_debug_infer_precision(self._h, int(precision), pi, po, n, _stream_ptr(stream)))

    # ---- configuration -----------------------------------------------------------------------
    def setStream(self, stream) -> None:
        check(self._lib.nrc_set_stream(self._h, _stream_ptr(stream)))

    def setHyperParams(self, hp: HyperParams) -> None:
        c = NrcHyperParams(float(hp.learningRate))
        check(self._lib.nrc_set_hyper_params(self._h, ctypes.byref(c)))

    def setConfig(self, encoding: InputEncoding) -> None:
        check(self._lib.nrc_set_config(self._h, int(encoding)))

    def getLearningRate(self) -> float:
        v = ctypes.c_float()
        check(self._lib.nrc_get_learning_rate(self._h, ctypes.byref(v)))
        return v.value

    def configJson(self) -> str:
        need = ctypes.c_size_t()
        check(self._lib.nrc_get_config_json(self._h, None, 0, ctypes.byref(need)))
        buf = ctypes.create_string_buffer(need.value)
        check(self._lib.nrc_get_config_json(self._h, buf, need.value, None))
        return buf.value.decode()

    set_stream = setStream
    set_hyper_params = setHyperParams
    set_config = setConfig
    get_learning_rate = getLearningRate
    config_json = configJson

    # ---- extensions: any batch size, data-parallel split, state ---------------------------
    def train_batch(self, inputs, targets, b: int, loss: bool = False):
        lh = ctypes.c_float(float("nan"))
        b = int(b)
        check(self._lib.nrc_train_batch(self._h, _dev_ptr(inputs, "inputs", b * self.query_dims if hasattr(inputs, "numel") else None),
                                        _dev_ptr(targets, "targets", b * 3 if hasattr(targets, "numel") else None), b,
                                        ctypes.byref(lh) if loss else None))
        return lh.value if loss else None

    def train_grad(self, inputs, targets, b: int, global_b: int, grad) -> None:
        b = int(b)
        check(self._lib.nrc_train_grad(self._h, _dev_ptr(inputs, "inputs", b * self.query_dims if hasattr(inputs, "numel") else None) if b else None,
                                       _dev_ptr(targets, "targets", b * 3 if hasattr(targets, "numel") else None) if b else None,
                                       b, int(global_b),
                                       _dev_ptr(grad, "grad", self.grad_floats if hasattr(grad, "numel") else None)))

    def train_apply(self, grad, loss: bool = False):
        lh = ctypes.c_float(float("nan"))
        check(self._lib.nrc_train_apply(self._h, _dev_ptr(grad, "grad", self.grad_floats if hasattr(grad, "numel") else None),
                                        ctypes.byref(lh) if loss else None))
        return lh.value if loss else None

    def train_grad_fixed(self, inputs, targets, b: int, global_b: int, grad, grid_fixed) -> None:
        """Hash only: nrc_train_grad with this rank's exact grid sums exchange-encoded into grid_fixed (int64,
        HASH_GRID_PARAMS; sum it over ranks as int64) and the grid part of grad left unwritten."""
        b = int(b)
        check(self._lib.nrc_train_grad_fixed(
            self._h, _dev_ptr(inputs, "inputs", b * self.query_dims if hasattr(inputs, "numel") else None) if b else None,
            _dev_ptr(targets, "targets", b * 3 if hasattr(targets, "numel") else None) if b else None, b, int(global_b),
            _dev_ptr(grad, "grad", self.grad_floats if hasattr(grad, "numel") else None),
            _dev_ptr(grid_fixed, "grid_fixed", HASH_GRID_PARAMS if hasattr(grid_fixed, "numel") else None,
                     "torch.int64")))

    def train_apply_fixed(self, grad, grid_fixed, loss: bool = False):
        """Hash only: the Adam + EMA step from the summed MLP gradient / loss in grad and the summed exact grid sums
        in grid_fixed (each rounded to f16 once)."""
        lh = ctypes.c_float(float("nan"))
        check(self._lib.nrc_train_apply_fixed(
            self._h, _dev_ptr(grad, "grad", self.grad_floats if hasattr(grad, "numel") else None),
            _dev_ptr(grid_fixed, "grid_fixed", HASH_GRID_PARAMS if hasattr(grid_fixed, "numel") else None,
                     "torch.int64"),
            ctypes.byref(lh) if loss else None))
        return lh.value if loss else None

    # ---- data parallelism inside the library (nrc_c.h: RCCL communicator + nrc_train_dp) ------------------
    def set_comm(self, comm) -> None:
        """Attach an RCCL communicator (a Communicator, an ncclComm_t address, or None to detach)."""
        c = comm.handle if isinstance(comm, Communicator) else comm
        check(self._lib.nrc_set_comm(self._h, c))

    def comm_rank(self) -> tuple[int, int]:
        r, w = ctypes.c_int(), ctypes.c_int()
        check(self._lib.nrc_get_comm_rank(self._h, ctypes.byref(r), ctypes.byref(w)))
        return r.value, w.value

    def train_dp(self, inputs, targets, b_local: int, global_b: int, loss: bool = False):
        """One data-parallel step: this rank's b_local samples of a global minibatch of global_b, the gradient
        all-reduced over the attached communicator inside the library, then the identical Adam + EMA step."""
        lh = ctypes.c_float(float("nan"))
        b = int(b_local)
        pi = _dev_ptr(inputs, "inputs", b * self.query_dims if hasattr(inputs, "numel") else None) if b else None
        pt = _dev_ptr(targets, "targets", b * 3 if hasattr(targets, "numel") else None) if b else None
        check(self._lib.nrc_train_dp(self._h, pi, pt, b, int(global_b), ctypes.byref(lh) if loss else None))
        return lh.value if loss else None

    def train_dp_async(self, inputs, targets, b_local: int, global_b: int, loss_d=None) -> None:
        """train_dp whose global loss goes to device memory (loss_d: a one-element f32 device tensor, or None);
        never blocks -- the form for one thread driving several in-process ranks (peer_exchange_open_local)."""
        b = int(b_local)
        pi = _dev_ptr(inputs, "inputs", b * self.query_dims if hasattr(inputs, "numel") else None) if b else None
        pt = _dev_ptr(targets, "targets", b * 3 if hasattr(targets, "numel") else None) if b else None
        pl = _dev_ptr(loss_d, "loss_d", 1 if hasattr(loss_d, "numel") else None) if loss_d is not None else None
        check(self._lib.nrc_train_dp_async(self._h, pi, pt, b, int(global_b), pl))

    # ---- one-shot peer exchange (nrc_c.h nrc_peer_exchange_*; round 4) --------------------------------------
    PEER_HANDLE_BYTES = 64

    def peer_exchange_handle(self, world: int) -> bytes:
        """Allocate this rank's receive buffer for a world of ranks; returns its IPC handle (64 bytes)."""
        buf = ctypes.create_string_buffer(self.PEER_HANDLE_BYTES)
        check(self._lib.nrc_peer_exchange_handle(self._h, int(world), buf))
        return buf.raw

    def peer_exchange_open(self, rank: int, world: int, handles: bytes) -> None:
        """Map every peer's receive buffer (handles: world x 64 bytes in rank order); train_dp then uses the exchange."""
        if len(handles) != int(world) * self.PEER_HANDLE_BYTES:
            raise ValueError("handles: world x 64 bytes in rank order")
        buf = ctypes.create_string_buffer(bytes(handles), len(handles))
        check(self._lib.nrc_peer_exchange_open(self._h, int(rank), int(world), buf))

    def peer_exchange_close(self) -> None:
        check(self._lib.nrc_peer_exchange_close(self._h))

    @staticmethod
    def peer_exchange_open_local(nets) -> None:
        """In-process peer exchange over several handles of this process (nrc_peer_exchange_open_local): nets[r] is
        rank r, the receive buffers are reached through plain device pointers. Close every handle before destroying
        any of them."""
        nets = list(nets)
        arr = (ctypes.c_void_p * len(nets))(*[n._h.value for n in nets])
        check(nets[0]._lib.nrc_peer_exchange_open_local(arr, len(nets)))

    def set_peer_seq(self, seq: int) -> None:
        """Test entry (nrc_debug_set_peer_seq): the sequence number of the last exchange step, between steps."""
        check(self._lib.nrc_debug_set_peer_seq(self._h, int(seq)))

    @property
    def num_params(self) -> int:
        """Parameter count of the configured model (Frequency 22,528; Hash 21,504 MLP + 991,232 grid)."""
        v = ctypes.c_uint64()
        check(self._lib.nrc_get_num_params(self._h, ctypes.byref(v)))
        return v.value

    @property
    def grad_floats(self) -> int:
        """Size of the data-parallel gradient buffer: num_params + 4 (the loss sits at index num_params)."""
        v = ctypes.c_uint64()
        check(self._lib.nrc_get_grad_floats(self._h, ctypes.byref(v)))
        return v.value

    def get_state(self, slot: StateSlot = StateSlot.PARAMS) -> np.ndarray:
        out = np.empty(self.num_params, dtype=np.float32)
        check(self._lib.nrc_get_state(self._h, int(slot), out.ctypes.data))
        return out

    def set_state(self, slot: StateSlot, values) -> None:
        v = np.ascontiguousarray(values, dtype=np.float32)
        n = self.num_params
        if v.size != n:
            raise ValueError(f"state must have {n} floats")
        check(self._lib.nrc_set_state(self._h, int(slot), v.ctypes.data))

    def encode_features(self, inputs, encoded, n: int, stream=None) -> None:
        """The production encoder of the configured encoding, f32 canonical order ([n][80]; Hash: [n][64] with the
        inference grid table)."""
        check(self._lib.nrc_debug_encode_net(self._h, _dev_ptr(inputs, "inputs"), _dev_ptr(encoded, "encoded"),
                                             int(n), _stream_ptr(stream)))

    @property
    def step(self) -> int:
        v = ctypes.c_uint32()
        check(self._lib.nrc_get_step(self._h, ctypes.byref(v)))
        return v.value

    @step.setter
    def step(self, value: int) -> None:
        check(self._lib.nrc_set_step(self._h, int(value)))


class Communicator:
    """An RCCL communicator made through the C-ABI helpers (nrc_comm_*): rank 0 calls unique_id(), shares the
    128 bytes with the other ranks (e.g. a torch.distributed broadcast), and every rank constructs one on its
    current HIP device."""

    UNIQUE_ID_BYTES = 128

    @staticmethod
    def unique_id() -> bytes:
        buf = ctypes.create_string_buffer(Communicator.UNIQUE_ID_BYTES)
        check(lib().nrc_comm_get_unique_id(buf))
        return buf.raw

    def __init__(self, unique_id: bytes, world: int, rank: int):
        if len(unique_id) != self.UNIQUE_ID_BYTES:
            raise ValueError("unique id must be 128 bytes")
        h = ctypes.c_void_p()
        check(lib().nrc_comm_init_rank(ctypes.byref(h), ctypes.create_string_buffer(unique_id, len(unique_id)),
                                       int(world), int(rank)))
        self.handle = h
        self.world, self.rank = int(world), int(rank)

    def destroy(self) -> None:
        if self.handle is not None and self.handle.value:
            check(lib().nrc_comm_destroy(self.handle))
            self.handle = ctypes.c_void_p()


def encode(inputs, encoded, n: int, stream=None) -> None:
    """The Composite encoding alone (test entry): f32 [n][80] canonical feature order."""
    check(lib().nrc_encode(_dev_ptr(inputs, "inputs"), _dev_ptr(encoded, "encoded"), int(n), _stream_ptr(stream)))


def default_config(encoding: InputEncoding = InputEncoding.Frequency, width: int = 64,
                   infer_precision: int = 0) -> NrcConfig:
    """The reference's hyper-parameters for an encoding; width 128 selects the BASELINE configs[4] network (f16
    training and inference), infer_precision PRECISION_FP8 its FP8 inference path (training stays f16);
    PRECISION_F16_ACC16 selects tiny-cuda-nn's f16-accumulate numerics for infer() (width 64, Frequency)."""
    c = lib().nrc_default_config(int(encoding))
    c.width = int(width)
    c.infer_precision = int(infer_precision)
    return c


def fp8_convert(x, y, n: int, relu: bool = True, stream=None) -> None:
    """e4m3 conversion exactly as the FP8 kernels do it (test entry): y[i] = e4m3(clamp(x[i], relu ? 0 : -448, 448))."""
    py = y if isinstance(y, int) else y.data_ptr()  # uint8 output
    if not isinstance(y, int) and (not y.is_cuda or y.numel() < n):
        raise ValueError("y: uint8 GPU tensor of >= n elements required")
    check(lib().nrc_debug_fp8_convert(_dev_ptr(x, "x", n), py, int(n), int(bool(relu)), _stream_ptr(stream)))


__all__ = ["Network", "Communicator", "InputEncoding", "HyperParams", "StateSlot", "NrcError", "encode", "default_config", "fp8_convert",
           "BATCH_SIZE", "NUM_PARAMS", "GRAD_FLOATS", "current_stream"]
