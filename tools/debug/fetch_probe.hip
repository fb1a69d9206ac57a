// fetch_probe.hip — calibrates rocprofv3 FETCH_SIZE for the parse kernel's
// access pattern (MI355X_MICROARCH.md §HBM: the x2 correction is calibrated
// for wide coalesced reads only).  A 1 GiB "text" with a line every 70-95
// bytes; two kernels read it:
//   probe_lines    one lane per line, the parse kernel's windows: 16-B loads
//                  at the line's aligned start +0/+16/+32/+48/+64 (the header
//                  and the read bases of a ~81-B line), offsets from an array
//   probe_stream   the same bytes as a coalesced 16-B-per-lane stream
//   probe_lines_w  probe_lines with the parse kernel's stores: 8 B (counts)
//                  and 16 B (header pair) per line
// Unique bytes: text + offsets (lines) / text (stream).  Run under
//   rocprofv3 --pmc FETCH_SIZE -- ./fetch_probe
// and compare FETCH_SIZE x 1024 (x 2?) with the printed byte counts.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                            \
        }                                                                            \
    } while (0)

__global__ __launch_bounds__(256) void probe_lines(const char* __restrict__ text, const uint64_t* __restrict__ starts,
                                                   uint64_t n, uint32_t* __restrict__ out)
{
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t a0 = starts[i] & ~(uint64_t)15;
        uint32_t x = 0;
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            const uint4 v = *(const uint4*)(text + a0 + 16 * k);
            x ^= v.x ^ v.y ^ v.z ^ v.w;
        }
        out[i] = x;
    }
}

__global__ __launch_bounds__(256) void probe_lines_w(const char* __restrict__ text,
                                                     const uint64_t* __restrict__ starts, uint64_t n,
                                                     uint64_t* __restrict__ c8, ulonglong2* __restrict__ h16)
{
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t a0 = starts[i] & ~(uint64_t)15;
        uint32_t x = 0, y = 0;
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            const uint4 v = *(const uint4*)(text + a0 + 16 * k);
            x ^= v.x ^ v.y;
            y ^= v.z ^ v.w;
        }
        c8[i] = ((uint64_t)y << 32) | x;
        h16[i] = make_ulonglong2(x, y);
    }
}

__global__ __launch_bounds__(256) void probe_stream(const uint4* __restrict__ text, uint64_t nq,
                                                    uint32_t* __restrict__ out)
{
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint32_t x = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nq; i += stride) {
        const uint4 v = text[i];
        x ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    out[(uint64_t)blockIdx.x * blockDim.x + threadIdx.x] = x;
}

int main()
{
    const uint64_t bytes = 1ull << 30, pad = 256;
    std::vector<char> h(bytes, 'A');
    std::vector<uint64_t> starts;
    uint64_t at = 0;
    uint32_t r = 12345;
    while (at + 100 < bytes) {
        starts.push_back(at);
        r = r * 1664525u + 1013904223u;
        at += 70 + (r >> 16) % 26;
        h[at - 1] = '\n';
    }
    const uint64_t n = starts.size();
    char* d_text;
    uint64_t* d_starts;
    uint32_t* d_out;
    CK(hipMalloc(&d_text, bytes + pad));
    CK(hipMalloc(&d_starts, n * 8));
    CK(hipMalloc(&d_out, std::max<uint64_t>(n, 1u << 20) * 4));
    uint64_t* d_c8;
    ulonglong2* d_h16;
    CK(hipMalloc(&d_c8, n * 8));
    CK(hipMalloc(&d_h16, n * 16));
    CK(hipMemcpy(d_text, h.data(), bytes, hipMemcpyHostToDevice));
    CK(hipMemset(d_text + bytes, 0, pad));
    CK(hipMemcpy(d_starts, starts.data(), n * 8, hipMemcpyHostToDevice));
    for (int rep = 0; rep < 3; ++rep) {
        probe_lines<<<16384, 256>>>(d_text, d_starts, n, d_out);
        probe_stream<<<4096, 256>>>((const uint4*)d_text, bytes / 16, d_out);
        probe_lines_w<<<16384, 256>>>(d_text, d_starts, n, d_c8, d_h16);
    }
    CK(hipDeviceSynchronize());
    std::printf("{\"lines\": %llu, \"text_bytes\": %llu, \"offset_bytes\": %llu, \"out_bytes_lines\": %llu}\n",
                (unsigned long long)n, (unsigned long long)bytes, (unsigned long long)(n * 8),
                (unsigned long long)(n * 4));
    return 0;
}
