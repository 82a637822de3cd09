"""oneccl_amd — MI355X-native local element-wise reduction for oneCCL.

Replaces the body of oneCCL's src/comp (ccl_comp_reduce and friends) with
hand-written CDNA4 HIP kernels behind a C ABI (include/mi_reduce.h), plus a
drop-in C++ shim keeping oneCCL's own signatures (include/mi_ccl_comp.h).
"""
from .comp import (  # noqa: F401
    DTYPE_SIZE,
    F_ACC_FP32,
    F_BF16_RNE,
    F_BF16_TAIL_TRUNC16,
    F_MINMAX_INOUT_FIRST,
    bf16_flags,
    bf16_impl,
    comp_batch_reduce,
    comp_copy,
    comp_reduce,
    datatype,
    env_reload,
    fp16_flags,
    fp16_impl,
    impl_types,
    reduce,
    reduce_multi,
    reduce_out,
    reduction,
    reduction_to_str,
    reference_flags,
    shard_range,
)

__version__ = "0.1.0"
