// aql_kernels.hip — code object for tools/aql_latency (built with --genco).
// An empty kernel and the lean 2-input fp32 sum, dispatched by raw AQL packets.
#include "../oneccl_amd/csrc/reduce_kernels.hpp"

extern "C" __global__ void aql_empty_kernel() {}

template __global__ void mi::reduce2_kernel<float, 0, 0u, 1, 1024>(mi::R2Args);
