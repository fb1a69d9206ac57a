// The VALU issue rate of one SIMD for the 32-bit integer instructions the
// tile parse and the writer are made of (v_add_u32, v_xor_b32, v_bitop3_b32,
// v_lshrrev_b32, v_and_or), measured: W waves a SIMD, each a stream of
// independent instructions (8 chains, unrolled), timed by HIP events and by
// the in-kernel clock (s_memtime against s_memrealtime's 100 MHz), so the
// cycles a wave64 instruction holds its SIMD come out with the clock the
// chip actually ran.  It sets bench.py's VALU_ISSUE_PER_S.
//   hipcc --offload-arch=gfx950 -O3 -o tools/debug/valu_rate_probe tools/debug/valu_rate_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr int ITERS = 4096;   // loop trips; each 8 chains x 4 ops = 32 VALU instructions

__global__ __launch_bounds__(256) void valu_stream(uint32_t* out, uint64_t* clk, uint32_t seed)
{
    uint32_t a[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = seed * (threadIdx.x + 17u * k + 1u);
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            uint32_t x = a[k];
            x = x + 0x7F7F7F7Fu;
            x ^= (x >> 7);
            x = (x & 0x0F0F0F0Fu) | (x >> 3);
            x = x + (uint32_t)i;
            a[k] = x;
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) s ^= a[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

int main()
{
    int dev = 0, cus = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    for (int blocks_per_cu : {1, 2, 4, 8}) {   // 256 threads: one wave a SIMD per block
        const int grid = cus * blocks_per_cu;
        uint32_t* out = nullptr;
        uint64_t* clk = nullptr;
        hipMalloc(&out, (size_t)grid * 256 * 4);
        hipMalloc(&clk, (size_t)grid * 16);
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        valu_stream<<<grid, 256>>>(out, clk, 3u);   // warm-up
        hipEventRecord(e0);
        valu_stream<<<grid, 256>>>(out, clk, 5u);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        uint64_t c[2] = {0, 0};
        hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost);
        // the VALU instructions a wave issues, counted from the code object
        // (ROCm 7.2 hipcc -O3: the loop unrolled twice, 96 VALU a trip:
        // v_add, v_lshrrev, v_xor, v_lshrrev, v_and_or per chain and step,
        // the i-adds folded into one scalar counter) -- recount if the
        // compiler changes
        constexpr double VALU_PER_WAVE = ITERS / 2 * 96.0;
        const double ghz = c[1] ? (double)c[0] / (double)c[1] * 0.1 : 0.0;
        const double wave_insts_per_simd = VALU_PER_WAVE * blocks_per_cu;
        const double cycles = ms * 1e-3 * ghz * 1e9;
        printf("{\"waves_per_simd\": %d, \"ms\": %.4f, \"clock_ghz\": %.3f, \"cycles_per_wave_inst_per_simd\": %.3f, "
               "\"note\": \"wave64 32-bit integer VALU, independent streams; cycles at the in-kernel clock\"}\n",
               blocks_per_cu, ms, ghz, cycles / wave_insts_per_simd);
        hipFree(out);
        hipFree(clk);
    }
    return 0;
}
