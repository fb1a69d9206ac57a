// Blocks a CU holds for a 256-thread kernel by its static LDS size
// (hipOccupancyMaxActiveBlocksPerMultiprocessor): the LDS allocation
// granule, which decides the tile parse's shapes (textpath.hip tp_halo).
#include <hip/hip_runtime.h>
#include <cstdio>
template <int B>
__global__ __launch_bounds__(256) void k(int* o)
{
    __shared__ char s[B];
    s[threadIdx.x] = (char)threadIdx.x;
    __syncthreads();
    o[threadIdx.x] = s[(threadIdx.x * 7) % B];
}
template <int B>
static void probe()
{
    int per = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k<B>, 256, 0) != hipSuccess) per = -1;
    printf("lds %6d B: %d blocks a CU\n", B, per);
}
int main()
{
    probe<20480>(); probe<23392>(); probe<23405>(); probe<23552>(); probe<24928>();
    probe<26624>(); probe<26976>(); probe<27136>(); probe<27306>(); probe<27307>(); probe<27488>();
    probe<31584>(); probe<32768>();
    return 0;
}
