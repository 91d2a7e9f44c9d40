// fpatomic_probe.hip — what gfx950's f64 atomics do with subnormals, infinities and rounding, as the collect kernels
// use them (-munsafe-fp-atomics: ds_add_f64 / global_atomic_add_f64).  The compensated flush (DESIGN §5 "Float
// parity") derives each addition's rounding error from the value the returning atomic saw; that is exact only if the
// atomic rounds to nearest-even like a VALU add, and keeps subnormals.
//   hipcc --offload-arch=gfx950 -O2 -munsafe-fp-atomics -ffp-contract=off tools/fpatomic_probe.hip -o tools/fpatomic_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <math.h>
#include <fenv.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 2; } } while (0)

// out[0..3]: LDS non-returning sum, LDS returning sum, global non-returning sum, global returning sum of the same lanes'
// values; out[4 + lane]: lane's returned old value (global); bad[0]: lanes whose old + v (VALU) != what the next
// returning atomic observed -- checked on the host from the returned sequence
__global__ void probe(const double* __restrict__ v, int n, double* out, double* olds_g, double* olds_l, double* g) {
    __shared__ double s[2];
    if (threadIdx.x == 0) { s[0] = 0.0; s[1] = 0.0; }
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        atomicAdd(&s[0], v[i]);
        olds_l[i] = atomicAdd(&s[1], v[i]);
        atomicAdd(&g[0], v[i]);
        olds_g[i] = atomicAdd(&g[1], v[i]);
    }
    __syncthreads();
    if (threadIdx.x == 0) { out[0] = s[0]; out[1] = s[1]; }
}

#pragma STDC FENV_ACCESS ON
static int run(const char* name, const double* hv, int n, int threads) {
    double *dv, *dout, *dog, *dol, *dg;
    CK(hipMalloc(&dv, n * 8)); CK(hipMalloc(&dout, 16)); CK(hipMalloc(&dog, n * 8)); CK(hipMalloc(&dol, n * 8));
    CK(hipMalloc(&dg, 16));
    CK(hipMemcpy(dv, hv, n * 8, hipMemcpyHostToDevice));
    CK(hipMemset(dg, 0, 16));
    hipLaunchKernelGGL(probe, dim3(1), dim3(threads), 0, 0, dv, n, dout, dog, dol, dg);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    double out[2], g[2];
    double* og = (double*)malloc(n * 8);
    double* ol = (double*)malloc(n * 8);
    CK(hipMemcpy(out, dout, 16, hipMemcpyDeviceToHost));
    CK(hipMemcpy(g, dg, 16, hipMemcpyDeviceToHost));
    CK(hipMemcpy(og, dog, n * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(ol, dol, n * 8, hipMemcpyDeviceToHost));
    // every returned old value is a prefix sum in the atomic's order: the set {old_i + v_i} must equal the set of
    // olds minus the first (0) plus the final value, if the atomic rounds like the VALU
    int bad_g = 0, bad_l = 0;
    for (int pass = 0; pass < 2; ++pass) {
        const double* o = pass ? ol : og;
        const double fin = pass ? out[1] : g[1];
        for (int i = 0; i < n; ++i) {
            const double s = o[i] + hv[i];
            bool found = memcmp(&s, &fin, 8) == 0;
            for (int k = 0; k < n && !found; ++k) found = memcmp(&s, &o[k], 8) == 0;
            if (!found) { if (pass) ++bad_l; else ++bad_g; }
        }
    }
    printf("%-22s lds=%a lds_rtn=%a glb=%a glb_rtn=%a  rtn-sequence mismatches: lds %d, global %d\n", name, out[0],
           out[1], g[0], g[1], bad_l, bad_g);
    // rounding mode of the atomic: the successor of each returned old value (the olds sorted by the order the atomic
    // applied them: for positive addends, ascending) against old + v rounded each way
    if (strcmp(name, "rounding 4096") == 0) {
        for (int pass = 0; pass < 2; ++pass) {
            double* o = pass ? ol : og;
            const double fin = pass ? out[1] : g[1];
            int* idx = (int*)malloc(n * sizeof(int));
            for (int i = 0; i < n; ++i) idx[i] = i;
            for (int i = 1; i < n; ++i) {  // insertion sort by old value
                int k = idx[i], j = i - 1;
                while (j >= 0 && o[idx[j]] > o[k]) { idx[j + 1] = idx[j]; --j; }
                idx[j + 1] = k;
            }
            int rn = 0, rz = 0, ru = 0, other = 0, exact = 0;
            for (int r = 0; r < n; ++r) {
                const int i = idx[r];
                const double next = r + 1 < n ? o[idx[r + 1]] : fin;
                fesetround(FE_TONEAREST); volatile double a = o[i]; volatile double b = hv[i]; const double sn = a + b;
                fesetround(FE_TOWARDZERO); const double sz = a + b;
                fesetround(FE_UPWARD); const double su = a + b;
                fesetround(FE_TONEAREST);
                if (sn == sz && sz == su) { ++exact; if (next != sn) ++other; continue; }
                if (next == sn) ++rn;
                if (next == sz) ++rz;
                if (next == su) ++ru;
                if (next != sn && next != sz && next != su) ++other;
            }
            printf("  %s atomic rounding: inexact adds matching RN %d, RZ %d, RU %d; exact adds %d; unexplained %d\n",
                   pass ? "lds" : "global", rn, rz, ru, exact, other);
            free(idx);
        }
    }
    free(og); free(ol);
    (void)hipFree(dv); (void)hipFree(dout); (void)hipFree(dog); (void)hipFree(dol); (void)hipFree(dg);
    return 0;
}

int main() {
    static double v[4096];
    const double tiny = ldexp(1.0, -1074), sub = ldexp(1.0, -1030);
    for (int i = 0; i < 64; ++i) v[i] = tiny;
    run("64 x 2^-1074", v, 64, 64);
    for (int i = 0; i < 64; ++i) v[i] = (i & 1) ? sub : -0.5 * sub;
    run("+-subnormals", v, 64, 64);
    v[0] = INFINITY; v[1] = 1.0; v[2] = -INFINITY; v[3] = 2.0;
    run("inf + -inf", v, 4, 4);
    v[0] = NAN; v[1] = 1.0;
    run("nan", v, 2, 2);
    v[0] = ldexp(1.0, 1023) * 1.9; v[1] = ldexp(1.0, 1023) * 1.9;
    run("overflow", v, 2, 1);
    // rounding: values with 53 significant bits of different magnitudes, one lane at a time (a known order)
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (int i = 0; i < 4096; ++i) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        v[i] = ldexp((double)(x >> 11), -53 + (int)(x % 40));
    }
    run("rounding 4096", v, 4096, 256);
    for (int i = 0; i < 4096; ++i) v[i] = (i & 3) == 0 ? 1e300 : ((i & 3) == 1 ? -1e300 : 1e-300 * i);
    run("cancel 4096", v, 4096, 256);
    return 0;
}
