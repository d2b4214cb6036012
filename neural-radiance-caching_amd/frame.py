"""Host-side mirror of the renderer's per-frame NRC steps around the network (include/nrc/frame.h).

These are the GPU steps the reference's ``Device`` launches after the OptiX trace
(/root/reference/nrc/src/Device.cpp:2493-2515):

===================================================  ==============================================
reference                                            here
===================================================  ==============================================
``accumulate_render_radiance`` (nrc_helpers.cu:77)   ``accumulate_render_radiance``
``copy_radiance_to_output_buffer`` (:54)             ``copy_radiance_to_output``
``propagate_train_radiance`` (:131)                  ``propagate_train_radiance``
``generateRandomPermutationForTrain`` (NRCUtil.cu)   ``generate_train_permutation``
``permute_train_data`` (:226)                        ``permute_train_data``
``Device::render`` post-trace sequence               ``process_frame``
===================================================  ==============================================

Buffers are device tensors (or raw addresses). Records use the reference's byte layout; on the host
they are numpy structured arrays (``TRAINING_RECORD_DTYPE``, ``END_VERTEX_DTYPE``) and on the device
int32 tensors of the same bytes (``records_to_device``).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from enum import IntEnum

import numpy as np

from ._lib import check, lib

NUM_TRAINING_RECORDS_PER_FRAME = 65536
NUM_BATCHES = 4
TRAIN_RECORD_INDEX_NONE = -1
TRAIN_RECORD_INDEX_BUFFER_FULL = -2

# TrainingRecord (neural_radiance_caching.h:57-75), 28 B
TRAINING_RECORD_DTYPE = np.dtype([("prop_to", "<i4"), ("local_throughput", "<f4", (3,)), ("pixel_index", "<i4"),
                                  ("tile_index", "<i4"), ("prop_length", "<i4")])
# TrainingSuffixEndVertex (neural_radiance_caching.h:78-94), 16 B
END_VERTEX_DTYPE = np.dtype([("start_train_record", "<i4"), ("radiance_mask", "<f4"), ("pixel_index", "<i4"),
                             ("tile_index", "<i4")])
assert TRAINING_RECORD_DTYPE.itemsize == 28 and END_VERTEX_DTYPE.itemsize == 16


class RenderMode(IntEnum):
    """nrc::RenderMode (neural_radiance_caching.h:14-22)."""
    Full = 0
    NoCache = 1
    CacheOnly = 2
    CacheFirstVertex = 3
    DebugCacheNoThroughputModulation = 4
    DebugThroughputOnly = 5


def _ptr(x, what: str) -> int | None:
    if x is None:
        return None
    if isinstance(x, int):
        return x
    if hasattr(x, "data_ptr"):
        if not x.is_cuda:
            raise ValueError(f"{what}: tensor must live on the GPU")
        if not x.is_contiguous():
            raise ValueError(f"{what}: tensor must be contiguous")
        return int(x.data_ptr())
    raise TypeError(f"{what}: expected a CUDA tensor or an integer device address, got {type(x)}")


def _stream(stream) -> int | None:
    if stream is None:
        return None
    if isinstance(stream, int):
        return stream
    return int(stream.cuda_stream)


def _sigs():
    L = lib()
    if getattr(L, "_frame_sigs", False):
        return L
    vp, u32, u64, i32, st = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int32, ctypes.c_int
    for name, args in {
        "nrc_accumulate_render_radiance": [vp, vp, vp, u32, ctypes.c_int, u32, vp],
        "nrc_copy_radiance_to_output": [vp, vp, u32, vp],
        "nrc_infer_accumulate": [vp, vp, vp, u32, vp, vp, u32, ctypes.c_int, u32],
        "nrc_propagate_train_radiance": [vp, vp, u32, vp, vp, u32, vp],
        "nrc_accumulate_render_radiance_factored": [vp, vp, vp, vp, u32, ctypes.c_int, u32, vp],
        "nrc_copy_radiance_to_output_factored": [vp, vp, vp, u32, vp],
        "nrc_propagate_train_radiance_factored": [vp, vp, vp, u32, vp, vp, vp, u32, vp],
        "nrc_generate_train_permutation": [u64, u32, vp, u32, vp],
        "nrc_sort_train_permutation": [vp, vp, vp, u32, vp, ctypes.c_size_t, vp],
        "nrc_permute_train_data": [vp, vp, vp, u64, u32, i32, vp, vp, u32, vp],
        "nrc_accumulate_render_radiance_factored_padded": [vp, vp, vp, vp, u32, ctypes.c_int, u32, vp],
        "nrc_copy_radiance_to_output_factored_padded": [vp, vp, vp, u32, vp],
        "nrc_propagate_train_radiance_factored_padded": [vp, vp, vp, u32, vp, vp, vp, u32, vp],
        "nrc_permute_train_data_padded": [vp, vp, vp, u64, u32, i32, vp, vp, u32, vp],
        "nrc_process_frame": [vp, ctypes.POINTER(NrcFrameBuffers), ctypes.POINTER(NrcFrameParams),
                              ctypes.POINTER(ctypes.c_float)],
        "nrc_process_frame_shard": [vp, ctypes.POINTER(NrcFrameBuffers), ctypes.POINTER(NrcFrameParams), u32, u32,
                                    ctypes.POINTER(ctypes.c_float)],
    }.items():
        fn = getattr(L, name)
        fn.restype = st
        fn.argtypes = args
    L._frame_sigs = True
    return L


class NrcFrameBuffers(ctypes.Structure):
    _fields_ = [("queries_inference_d", ctypes.c_void_p), ("results_inference_d", ctypes.c_void_p),
                ("last_render_throughput_d", ctypes.c_void_p), ("output_rgba_d", ctypes.c_void_p),
                ("queries_cache_vis_d", ctypes.c_void_p), ("results_cache_vis_d", ctypes.c_void_p),
                ("end_vertices_d", ctypes.c_void_p), ("train_records_d", ctypes.c_void_p),
                ("train_queries_d", ctypes.c_void_p * 2), ("train_targets_d", ctypes.c_void_p * 2),
                ("permutation_d", ctypes.c_void_p), ("shuffle_keys_d", ctypes.c_void_p)]


class NrcFrameParams(ctypes.Structure):
    _fields_ = [("screen_size", ctypes.c_uint32), ("num_tiles", ctypes.c_uint32),
                ("num_training_records", ctypes.c_int32), ("render_mode", ctypes.c_int32),
                ("iteration_index", ctypes.c_uint32), ("frame_index", ctypes.c_uint32),
                ("shuffle_seed", ctypes.c_uint64), ("train", ctypes.c_int32), ("keep_render_results", ctypes.c_int32),
                ("reflectance_factoring", ctypes.c_int32)]


def accumulate_render_radiance(radiance, throughput, output_rgba, num_pixels: int, mode: RenderMode,
                               iteration_index: int, stream=None) -> None:
    check(_sigs().nrc_accumulate_render_radiance(_ptr(radiance, "radiance"), _ptr(throughput, "throughput"),
                                                 _ptr(output_rgba, "output_rgba"), int(num_pixels), int(mode),
                                                 int(iteration_index), _stream(stream)))


def accumulate_render_radiance_factored(radiance, queries, throughput, output_rgba, num_pixels: int, mode: RenderMode,
                                        iteration_index: int, stream=None, padded: bool = False) -> None:
    """USE_REFLECTANCE_FACTORING 1 form (frame.h): the radiance times the render query's reflectance (padded: the
    queries are 16-float records, USE_COMPACT_RADIANCE_QUERY 0)."""
    fn = _sigs().nrc_accumulate_render_radiance_factored_padded if padded else _sigs().nrc_accumulate_render_radiance_factored
    check(fn(_ptr(radiance, "radiance"), _ptr(queries, "queries"), _ptr(throughput, "throughput"),
             _ptr(output_rgba, "output_rgba"), int(num_pixels), int(mode), int(iteration_index), _stream(stream)))


def propagate_train_radiance_factored(end_vertices, end_radiance, end_queries, num_tiles: int, records, targets,
                                      train_queries, num_records: int, stream=None, padded: bool = False) -> None:
    """USE_REFLECTANCE_FACTORING 1 form of propagate_train_radiance (frame.h): targets hold radiance / reflectance."""
    fn = _sigs().nrc_propagate_train_radiance_factored_padded if padded else _sigs().nrc_propagate_train_radiance_factored
    check(fn(_ptr(end_vertices, "end_vertices"), _ptr(end_radiance, "end_radiance"), _ptr(end_queries, "end_queries"),
             int(num_tiles), _ptr(records, "records"), _ptr(targets, "targets"), _ptr(train_queries, "train_queries"),
             int(num_records), _stream(stream)))


def infer_accumulate(net, queries, results, n: int, throughput, output_rgba, num_pixels: int, mode: RenderMode,
                     iteration_index: int) -> None:
    """infer() with accumulate_render_radiance fused into its epilogue for the render queries [0, num_pixels)
    (their radiance is not written to ``results``); on the network's stream."""
    check(_sigs().nrc_infer_accumulate(net._h, _ptr(queries, "queries"), _ptr(results, "results"), int(n),
                                       _ptr(throughput, "throughput"), _ptr(output_rgba, "output_rgba"),
                                       int(num_pixels), int(mode), int(iteration_index)))


def copy_radiance_to_output(radiance, output_rgba, num_pixels: int, stream=None) -> None:
    check(_sigs().nrc_copy_radiance_to_output(_ptr(radiance, "radiance"), _ptr(output_rgba, "output_rgba"),
                                              int(num_pixels), _stream(stream)))


def propagate_train_radiance(end_vertices, end_radiance, num_tiles: int, records, targets, num_records: int,
                             stream=None) -> None:
    check(_sigs().nrc_propagate_train_radiance(_ptr(end_vertices, "end_vertices"), _ptr(end_radiance, "end_radiance"),
                                               int(num_tiles), _ptr(records, "records"), _ptr(targets, "targets"),
                                               int(num_records), _stream(stream)))


def generate_train_permutation(seed: int, frame_index: int, permutation, n: int, stream=None) -> None:
    check(_sigs().nrc_generate_train_permutation(int(seed), int(frame_index), _ptr(permutation, "permutation"),
                                                 int(n), _stream(stream)))


def sort_train_permutation_temp_bytes(n: int) -> int:
    L = lib()
    fn = L.nrc_sort_train_permutation_temp_bytes
    fn.restype, fn.argtypes = ctypes.c_size_t, [ctypes.c_uint32]
    return int(fn(int(n)))


def sort_train_permutation(keys, permutation, n: int, sorted_keys=None, temp=None, stream=None) -> None:
    """The reference's shuffle (NRCUtil.cu:19-35): permutation[0:n] = the indices of a stable sort of the u32 keys
    (cub::DeviceRadixSort::SortPairs(keys, iota)); sorted_keys (optional) = the sorted keys. Device tensors of 4-byte
    elements; temp: a device buffer of sort_train_permutation_temp_bytes(n) bytes (allocated here if None)."""
    if temp is None:
        import torch
        temp = torch.empty(max(1, sort_train_permutation_temp_bytes(n)), dtype=torch.uint8, device=keys.device)
    nbytes = temp.numel() * temp.element_size() if hasattr(temp, "numel") else sort_train_permutation_temp_bytes(n)
    check(_sigs().nrc_sort_train_permutation(_ptr(keys, "keys"), _ptr(sorted_keys, "sorted_keys"),
                                             _ptr(permutation, "permutation"), int(n), _ptr(temp, "temp"), int(nbytes),
                                             _stream(stream)))


def permute_train_data(queries_src, targets_src, permutation, seed: int, frame_index: int, num_records: int,
                       queries_dst, targets_dst, n_out: int = NUM_TRAINING_RECORDS_PER_FRAME, stream=None,
                       padded: bool = False) -> None:
    fn = _sigs().nrc_permute_train_data_padded if padded else _sigs().nrc_permute_train_data
    check(fn(_ptr(queries_src, "queries_src"), _ptr(targets_src, "targets_src"), _ptr(permutation, "permutation"),
             int(seed), int(frame_index), int(num_records), _ptr(queries_dst, "queries_dst"),
             _ptr(targets_dst, "targets_dst"), int(n_out), _stream(stream)))


def records_to_device(arr: np.ndarray, device):
    """Structured host records -> int32 device tensor holding the same bytes."""
    import torch
    a = np.ascontiguousarray(arr)
    return torch.from_numpy(a.view(np.int32).reshape(len(a), a.dtype.itemsize // 4).copy()).to(device)


def records_from_device(t, dtype: np.dtype) -> np.ndarray:
    return np.ascontiguousarray(t.cpu().numpy()).view(dtype).reshape(-1)


@dataclass
class FrameBuffers:
    """Device buffers of one frame, as the reference's ControlBlock holds them (neural_radiance_caching.h:126-187).
    Capacity of the inference buffers is screen + max tiles (Device.cpp:1246-1253)."""
    queries_inference: object
    results_inference: object
    last_render_throughput: object
    output_rgba: object
    end_vertices: object
    train_records: object
    train_queries: list
    train_targets: list
    queries_cache_vis: object = None
    results_cache_vis: object = None
    permutation: object = None
    shuffle_keys: object = None  # u32 keys (any 4-byte dtype) whose stable sort is the permutation (frame.h)
    _keep: list = field(default_factory=list)

    def as_struct(self) -> NrcFrameBuffers:
        fb = NrcFrameBuffers()
        fb.queries_inference_d = _ptr(self.queries_inference, "queries_inference")
        fb.results_inference_d = _ptr(self.results_inference, "results_inference")
        fb.last_render_throughput_d = _ptr(self.last_render_throughput, "last_render_throughput")
        fb.output_rgba_d = _ptr(self.output_rgba, "output_rgba")
        fb.queries_cache_vis_d = _ptr(self.queries_cache_vis, "queries_cache_vis")
        fb.results_cache_vis_d = _ptr(self.results_cache_vis, "results_cache_vis")
        fb.end_vertices_d = _ptr(self.end_vertices, "end_vertices")
        fb.train_records_d = _ptr(self.train_records, "train_records")
        fb.train_queries_d[0] = _ptr(self.train_queries[0], "train_queries[0]")
        fb.train_queries_d[1] = _ptr(self.train_queries[1], "train_queries[1]")
        fb.train_targets_d[0] = _ptr(self.train_targets[0], "train_targets[0]")
        fb.train_targets_d[1] = _ptr(self.train_targets[1], "train_targets[1]")
        fb.permutation_d = _ptr(self.permutation, "permutation")
        fb.shuffle_keys_d = _ptr(self.shuffle_keys, "shuffle_keys")
        return fb


@dataclass
class FrameParams:
    screen_size: int
    num_tiles: int
    num_training_records: int
    render_mode: RenderMode = RenderMode.Full
    iteration_index: int = 0
    frame_index: int = 0
    shuffle_seed: int = 0
    train: bool = True
    keep_render_results: bool = False
    reflectance_factoring: bool = False

    def as_struct(self) -> NrcFrameParams:
        return NrcFrameParams(int(self.screen_size), int(self.num_tiles), int(self.num_training_records),
                              int(self.render_mode), int(self.iteration_index), int(self.frame_index),
                              int(self.shuffle_seed), int(bool(self.train)), int(bool(self.keep_render_results)),
                              int(bool(self.reflectance_factoring)))


def process_frame(net, buffers: FrameBuffers, params: FrameParams, loss: bool = True):
    """Device::render's post-trace NRC sequence for one frame (Device.cpp:2493-2515) on the network's stream:
    infer -> accumulate (or cache-vis) -> propagate -> shuffle -> 4 x train. Returns the mean minibatch
    loss if ``loss`` (blocking), else None."""
    fb, fp = buffers.as_struct(), params.as_struct()
    lh = ctypes.c_float(float("nan"))
    check(_sigs().nrc_process_frame(net._h, ctypes.byref(fb), ctypes.byref(fp), ctypes.byref(lh) if loss else None))
    return lh.value if loss else None


def process_frame_shard(net, buffers: FrameBuffers, params: FrameParams, pixel_begin: int, pixel_end: int,
                        loss: bool = True):
    """Data-parallel replica of process_frame (frame.h nrc_process_frame_shard): renders pixels [pixel_begin,
    pixel_end), infers every train-suffix end, and with a communicator attached trains on this rank's slice of
    every minibatch through nrc_train_dp."""
    fb, fp = buffers.as_struct(), params.as_struct()
    lh = ctypes.c_float(float("nan"))
    check(_sigs().nrc_process_frame_shard(net._h, ctypes.byref(fb), ctypes.byref(fp), int(pixel_begin), int(pixel_end),
                                          ctypes.byref(lh) if loss else None))
    return lh.value if loss else None
