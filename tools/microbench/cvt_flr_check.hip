// cvt_flr_check.hip -- exhaustive check of v_cvt_flr_i32_f32 against (int)floorf on gfx950, over every
// finite float whose floor fits in int32 (all 2^32 bit patterns are visited; NaN / inf / out-of-range
// values are skipped).  The padded-leaf-map general-view march (vr_kernels.hip, f.pad) converts
// positions with it.  Prints the number of mismatches and the first one.
//   hipcc --offload-arch=gfx950 -O3 cvt_flr_check.hip -o /tmp/cvt_flr_check && /tmp/cvt_flr_check
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>

__global__ void check(unsigned long long base, unsigned long long* bad, unsigned* first) {
    const unsigned long long i = base + (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > 0xffffffffull) return;
    const float x = __uint_as_float((unsigned)i);
    if (!(fabsf(x) < 2147483520.0f)) return;   // NaN, inf, or a floor outside int32
    int r;
    asm volatile("v_cvt_flr_i32_f32 %0, %1" : "=v"(r) : "v"(x));
    const int e = (int)floorf(x);
    if (r != e) {
        atomicAdd(bad, 1ull);
        atomicMin(first, (unsigned)i);
    }
}

int main() {
    unsigned long long* bad;
    unsigned* first;
    hipMalloc(&bad, 8);
    hipMalloc(&first, 4);
    hipMemset(bad, 0, 8);
    hipMemset(first, 0xff, 4);
    const unsigned long long chunk = 1ull << 30;
    for (unsigned long long b = 0; b < (1ull << 32); b += chunk)
        hipLaunchKernelGGL(check, dim3((unsigned)(chunk / 256)), dim3(256), 0, 0, b, bad, first);
    unsigned long long h = 0;
    unsigned f = 0;
    hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost);
    hipMemcpy(&f, first, 4, hipMemcpyDeviceToHost);
    if (hipGetLastError() != hipSuccess) { printf("hip error\n"); return 2; }
    printf("{\"mismatches\": %llu, \"first_bits\": \"0x%08x\"}\n", h, f);
    return h ? 1 : 0;
}
