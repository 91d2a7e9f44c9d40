// Diagnostic (not part of the library): is config 4's floored stream bound by the hashing (VALU) or by the loads?
// Times, over n 8-byte values: the loads alone, the mix64 hash + floor test alone (values from the index), and both.
//   hipcc -O3 --offload-arch=gfx950 tools/hashbench.hip -o tools/hashbench && tools/hashbench 125000000
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); std::exit(1); } } while (0)

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 32)) * 0x4cd6944c5cc20b6dULL;
    z = (z ^ (z >> 29)) * 0xfc12c5b19d3259e9ULL;
    return z ^ (z >> 32);
}

template <int MODE>  // 0 loads, 1 hash, 2 loads + hash
__global__ __launch_bounds__(1024) void bench(const uint64_t* __restrict__ v, uint64_t n, uint64_t zmask,
                                              unsigned long long* out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * 4;
    unsigned long long acc = 0;
    for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n; i += stride) {
        uint64_t x[4];
        if (MODE != 1) {
            const ulonglong2* p = (const ulonglong2*)(v + i);
            const ulonglong2 a = p[0], b = p[1];
            x[0] = a.x; x[1] = a.y; x[2] = b.x; x[3] = b.y;
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) x[j] = (i + j) * 0x9E3779B97F4A7C15ULL;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (MODE == 0) acc += x[j];
            else acc += (mix64(x[j]) & zmask) == 0;
        }
    }
    if (acc == 0x5555) atomicAdd(out, acc);  // keeps the work; never taken in practice
}

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 125000000ull;
    uint64_t* v;
    unsigned long long* out;
    CK(hipMalloc(&v, n * 8));
    CK(hipMalloc(&out, 8));
    CK(hipMemset(v, 1, n * 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const uint64_t zmask = ((1ull << 9) - 1) << (64 - 18 - 9);
    for (int blocks : {512, 1024, 2048, 4096}) {
        for (int mode = 0; mode < 3; ++mode) {
            float best = 1e9f;
            for (int r = 0; r < 8; ++r) {
                CK(hipEventRecord(e0));
                if (mode == 0) hipLaunchKernelGGL(bench<0>, dim3(blocks), dim3(1024), 0, 0, v, n, zmask, out);
                if (mode == 1) hipLaunchKernelGGL(bench<1>, dim3(blocks), dim3(1024), 0, 0, v, n, zmask, out);
                if (mode == 2) hipLaunchKernelGGL(bench<2>, dim3(blocks), dim3(1024), 0, 0, v, n, zmask, out);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (r > 0 && ms < best) best = ms;
            }
            std::printf("blocks %5d  %-12s %8.1f us  %7.1f GB/s\n", blocks,
                        mode == 0 ? "loads" : mode == 1 ? "hash" : "loads+hash", best * 1e3, n * 8 / (best * 1e-3) / 1e9);
        }
    }
    return 0;
}
