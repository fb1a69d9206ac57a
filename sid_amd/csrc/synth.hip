// synth.hip — device side of the counter-based synthetic pileup (synth.h).
// Fills profile_t counts for sites [first, first+n) directly in HBM, so the
// bench's inputs are resident before the timed region starts.
#include <hip/hip_runtime.h>

#include "synth.h"

namespace {
__global__ __launch_bounds__(256) void sid_synth_kernel(uint64_t seed, uint64_t first, size_t n,
                                                        const uint64_t* __restrict__ cdf,
                                                        uint32_t kmax, uint64_t* __restrict__ out)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        out[i] = sid_synth_counts(seed, first + i, cdf, kmax);
}
}  // namespace

extern "C" hipError_t sid_launch_synth(uint64_t seed, uint64_t first, size_t n,
                                       const uint64_t* d_cdf, uint32_t kmax, uint16_t* counts,
                                       hipStream_t stream)
{
    if (n == 0) return hipSuccess;
    size_t want = (n + 255) / 256;
    int grid = (int)(want < 8192 ? want : 8192);
    sid_synth_kernel<<<grid, 256, 0, stream>>>(seed, first, n, d_cdf, kmax, (uint64_t*)counts);
    return hipGetLastError();
}
