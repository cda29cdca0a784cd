// Dev: the achievable HBM ceiling of the Jacobian sweep's traffic pattern.
// The same bytes as sweep_kernel<5,true,32,2> at B instances — per instance 304 B read, 3968 B written — moved by an
// ideal streaming kernel: chunks of 32 instances per wave (as the sweep), the chunk's inputs read once into registers,
// its output block written front to back with 16-byte stores by all 64 lanes (1 KiB per store instruction), a
// grid-stride loop over the chunks on a persistent grid.  No arithmetic, no LDS: only the traffic.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o tools/_sweep_ceiling.so tools/sweep_ceiling.hip
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {
constexpr int CH = 32;                     // instances per chunk (one wave)
constexpr int IN16 = CH * 304 / 16;        // 608 16-byte input words per chunk
constexpr int OUT16 = CH * 3968 / 16;      // 7936 16-byte output words per chunk
constexpr int IN_PER_LANE = (IN16 + 63) / 64;   // 10
constexpr int OUT_PER_LANE = OUT16 / 64;        // 124

__global__ __launch_bounds__(128) void stream_kernel(const double2* __restrict__ in, double2* __restrict__ out,
                                                     long long nchunk)
{
    const int lane = threadIdx.x & 63;
    const long long w0 = (long long)blockIdx.x * 2 + (threadIdx.x >> 6);
    const long long stride = (long long)gridDim.x * 2;
    for (long long c = w0; c < nchunk; c += stride) {
        double2 r[IN_PER_LANE];
        const double2* ic = in + c * IN16;
#pragma unroll
        for (int j = 0; j < IN_PER_LANE; ++j) {
            const int e = lane + 64 * j;
            r[j] = e < IN16 ? ic[e] : make_double2(0.0, 0.0);
        }
        double2* oc = out + c * OUT16;
#pragma unroll 4
        for (int k = 0; k < OUT_PER_LANE; ++k) {
            const double2 v = r[k % IN_PER_LANE];
            oc[lane + 64 * k] = make_double2(v.x + (double)k, v.y);
        }
    }
}

// r6: the same bytes in the runtime fill's order — the grid as a whole streams each buffer front to
// back: store instruction k of wave w writes 1 KiB slice k * waves + w, so the grid's concurrent stores hit consecutive
// slices (few open DRAM pages) instead of one 124 KiB block per wave; 256-thread workgroups, up to 8 per CU (32 waves).
__global__ __launch_bounds__(256) void fill_order_kernel(const double2* __restrict__ in, double2* __restrict__ out,
                                                         long long n_in16, long long n_out16)
{
    const int lane = threadIdx.x & 63;
    const long long w = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    const long long waves = (long long)gridDim.x * 4;
    double2 acc = make_double2(0.0, 0.0);
    for (long long e = w * 64 + lane; e < n_in16; e += waves * 64) {
        const double2 v = in[e];
        acc.x += v.x;
        acc.y += v.y;
    }
#pragma unroll 4
    for (long long e = w * 64 + lane; e < n_out16; e += waves * 64) out[e] = make_double2(acc.x + (double)e, acc.y);
}
}  // namespace

extern "C" int fill_order_launch(const void* in, void* out, long long B, int grid, void* stream)
{
    hipLaunchKernelGGL(fill_order_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const double2*)in,
                       (double2*)out, B * 304 / 16, B * 3968 / 16);
    return (int)hipGetLastError();
}

extern "C" int fill_order_resident(int* blocks)
{
    int per_cu = 0, dev = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fill_order_kernel, 256, 0) != hipSuccess) return -1;
    if (hipGetDevice(&dev) != hipSuccess) return -1;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return -1;
    *blocks = per_cu * cus;
    return 0;
}

extern "C" int ceiling_launch(const void* in, void* out, long long B, int grid, void* stream)
{
    if (B % CH) return -1;
    hipLaunchKernelGGL(stream_kernel, dim3(grid), dim3(128), 0, (hipStream_t)stream, (const double2*)in,
                       (double2*)out, B / CH);
    return (int)hipGetLastError();
}

extern "C" int ceiling_resident(int* blocks)
{
    int per_cu = 0, dev = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, stream_kernel, 128, 0) != hipSuccess) return -1;
    if (hipGetDevice(&dev) != hipSuccess) return -1;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return -1;
    *blocks = per_cu * cus;
    return 0;
}
