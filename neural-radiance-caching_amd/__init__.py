"""MI355X-native neural radiance cache: drop-in for the reference's nrc::Network query/train module.

Product = libnrc_amd.so (hand-written gfx950 HIP kernels behind the C-ABI in include/nrc/nrc_c.h).
This package is the host-side mirror of the reference interface plus the synthetic Cornell sample
stream and the data-parallel sharding. The directory name contains hyphens, so it is loaded as the
module ``nrc_amd`` by ``load()`` in __graft_entry__.py / tests/conftest.py / bench.py.
"""
from . import _lib, dp, frame, stream, synthetic  # noqa: F401
from ._lib import (BATCH_SIZE, FIXED_MAX_RANKS, GRAD_FLOATS, HASH_GRAD_FLOATS, HASH_GRID_PARAMS,  # noqa: F401
                   HASH_MLP_PARAMS, HASH_NUM_PARAMS, NUM_PARAMS, NrcError)
from ._lib import PRECISION_F16, PRECISION_F16_ACC16, PRECISION_FP8, QUERY_COMPACT, QUERY_PADDED, WIDE_NUM_PARAMS  # noqa: F401
from .network import (Communicator, HyperParams, InputEncoding, Network, StateSlot, current_stream, default_config, encode,  # noqa: F401
                      fp8_convert)
