// Kernels either side of the march: the synthetic C5 volume generator and frame
// egress to display-ordered RGB8 (myApp.cu:1661-1688 point list, the 180 degree
// VRC rotation of myApp.cu:933 and stbi's vertical flip, myApp.cu:1954).  Both are HBM-streaming:
// one pass, coalesced along the fastest output axis.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "vr_device.h"

#pragma clang fp contract(off)

namespace vr {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// v(x,y,z) for an n^3 volume; same double-precision expression order as oracle or_synthetic_voxel.
// One block row per (x, y) line: threads walk z, so stores are contiguous.
__global__ void __launch_bounds__(256) synthetic_kernel(float* __restrict__ out, int64_t n, int64_t x0, int64_t nx,
                                                        uint64_t seed) {
    const double c = (double)(n - 1) / 2.0, half = (double)n / 2.0;
    const int64_t lines = nx * n;
    for (int64_t line = blockIdx.x; line < lines; line += gridDim.x) {
        const int64_t x = x0 + line / n, y = line % n;
        const double dx = (double)x - c, dy = (double)y - c;
        const double dxy = dx * dx + dy * dy;
        float* row = out + line * n;
        for (int64_t z = threadIdx.x; z < n; z += blockDim.x) {
            const double dz = (double)z - c;
            const double r = sqrt(dxy + dz * dz) / half;
            float v = 0.0f;
            if (r < 0.95) {
                const double w = round(127.5 + 127.5 * sin(16.0 * M_PI * r));
                const int64_t idx = (x * n + y) * n + z;
                const int64_t noise = (int64_t)(splitmix64(seed ^ (uint64_t)idx) % 17u) - 8;
                int64_t iv = (int64_t)w + noise;
                iv = iv < 0 ? 0 : (iv > 255 ? 255 : iv);
                v = (float)iv;
            }
            row[z] = v;
        }
    }
}

hipError_t launch_synthetic(float* out, int64_t n, int64_t x0, int64_t nx, uint64_t seed, hipStream_t st) {
    const int64_t lines = nx * n;
    if (lines == 0) return hipSuccess;
    const unsigned grid = (unsigned)(lines < 65536 ? lines : 65536);
    hipLaunchKernelGGL(synthetic_kernel, dim3(grid), dim3(256), 0, st, out, n, x0, nx, seed);
    return hipGetLastError();
}

// float RGBA frame [x*H + y] -> RGB8 image rows, quantised like a GL unorm8 framebuffer
// (round(clamp(c) * 255)).  orient 0: img[y][x]; 1 (VRC display): img[y][W-1-x];
// 2 (TEST display): img[H-1-y][x].  One thread per output pixel, row-major: coalesced stores,
// strided (stride 16*H B) but cache-line-shared reads across the 64 y-adjacent lanes of a column.
__global__ void __launch_bounds__(256) egress_kernel(const float4* __restrict__ frame, uint8_t* __restrict__ rgb,
                                                     int W, int H, int orient) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)W * H) return;
    const int r = (int)(i / W), col = (int)(i % W);
    int x, y;
    if (orient == 1) { x = W - 1 - col; y = r; }
    else if (orient == 2) { x = col; y = H - 1 - r; }
    else { x = col; y = r; }
    const float4 f = frame[(int64_t)x * H + y];
    const float ch[3] = {f.x, f.y, f.z};
    for (int k = 0; k < 3; ++k) {
        const float v = fminf(fmaxf(ch[k], 0.0f), 1.0f);
        rgb[i * 3 + k] = (uint8_t)rintf(v * 255.0f);
    }
}

hipError_t launch_egress(const float4* frame, uint8_t* rgb, int W, int H, int orient, hipStream_t st) {
    const int64_t n = (int64_t)W * H;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(egress_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, frame, rgb, W, H, orient);
    return hipGetLastError();
}

// POINT mode (prepareVolumeColors, myApp.cu:1280-1316): 7 floats per voxel, the GL vertex layout
// [x y z r g b a] at voxel index (x*d2 + y)*d3 + z.  Position ((v + L/2) - d/2) / L in float, colour
// TF(volume / cal_max) with the division in double (float -> getMaterial(float)).  Each workgroup
// builds its 256 x 7 floats in LDS and stores them as contiguous float4s (28 B per voxel would
// otherwise be written by 7 strided store instructions).
__global__ void __launch_bounds__(256) point_kernel(const float* __restrict__ vol, int64_t n, int64_t d2, int64_t d3,
                                                    float vd0, float vd1, float vd2, int L, double cal_max,
                                                    const float* __restrict__ lo, const float* __restrict__ hi,
                                                    int n_tf, const float4* __restrict__ rgba,
                                                    float* __restrict__ out) {
    __shared__ float s_lo[kMaxTf], s_hi[kMaxTf];
    __shared__ float4 s_rgba[kMaxTf];
    __shared__ __attribute__((aligned(16))) float s_out[256 * 7];
    for (int i = threadIdx.x; i < n_tf; i += blockDim.x) { s_lo[i] = lo[i]; s_hi[i] = hi[i]; s_rgba[i] = rgba[i]; }
    __syncthreads();
    const float hL = L / 2.0f, fL = (float)L;
    for (int64_t base = (int64_t)blockIdx.x * 256; base < n; base += (int64_t)gridDim.x * 256) {
        const int64_t i = base + threadIdx.x;
        if (i < n) {
            const int64_t x = i / (d2 * d3), y = (i / d3) % d2, z = i % d3;
            float* o = s_out + threadIdx.x * 7;
            o[0] = (((float)x + hL) - (vd0 / 2.0f)) / fL;
            o[1] = (((float)y + hL) - (vd1 / 2.0f)) / fL;
            o[2] = (((float)z + hL) - (vd2 / 2.0f)) / fL;
            const float4 c = s_rgba[tf_class(s_lo, s_hi, n_tf, (float)((double)vol[i] / cal_max))];
            o[3] = c.x; o[4] = c.y; o[5] = c.z; o[6] = c.w;
        }
        __syncthreads();
        const int64_t cnt = (n - base < 256 ? n - base : 256) * 7;   // floats of this block
        float* dst = out + base * 7;                                  // 16-B aligned: base*28 = k*7168
        const int64_t n4 = cnt / 4;
        for (int64_t k = threadIdx.x; k < n4; k += blockDim.x)
            reinterpret_cast<float4*>(dst)[k] = reinterpret_cast<const float4*>(s_out)[k];
        for (int64_t k = n4 * 4 + threadIdx.x; k < cnt; k += blockDim.x) dst[k] = s_out[k];
        __syncthreads();
    }
}

hipError_t launch_point(const float* vol, int64_t d1, int64_t d2, int64_t d3, double cal_max, const float* lo,
                        const float* hi, int n_tf, const float4* rgba, float* out, hipStream_t st) {
    const int64_t n = d1 * d2 * d3;
    if (n == 0) return hipSuccess;
    int64_t L = d1 > d2 ? d1 : d2;
    L = L > d3 ? L : d3;
    const int64_t blocks64 = (n + 255) / 256;
    const unsigned grid = (unsigned)(blocks64 < 65536 ? blocks64 : 65536);
    hipLaunchKernelGGL(point_kernel, dim3(grid), dim3(256), 0, st, vol, n, d2, d3, (float)d1, (float)d2, (float)d3,
                       (int)L, cal_max, lo, hi, n_tf, rgba, out);
    return hipGetLastError();
}

}  // namespace vr
