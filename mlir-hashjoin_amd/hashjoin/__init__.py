"""hashjoin -- MI355X-native hash-join operator (host side).

Python view of libhj.so (include/hj.h).  The join itself is hand-written HIP
for gfx950 in ../csrc; this package only plumbs device tensors, streams and
torch.distributed around it.  Importing fails loudly when libhj.so is
missing: there is no CPU fallback.
"""
from ._lib import HJError, check, declared_symbols, lib  # noqa: F401
from .join import (HashJoin, device_info, gen_pkfk, gen_uniform_i32, gen_uniform_i64, gen_zipf,  # noqa: F401
                   hit_threshold, partition_of, placement_stats, stream_copy, zipf_params)

__all__ = ["HashJoin", "device_info", "HJError", "gen_pkfk", "gen_uniform_i32", "gen_uniform_i64", "hit_threshold",
           "partition_of", "placement_stats", "stream_copy", "gen_zipf", "zipf_params", "lib", "check", "declared_symbols"]
