// vr_march.h -- device helpers shared by the march kernels (vr_kernels.hip: VRC and the setup
// kernels; vr_test.hip: TEST).  Internal, not the ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "vr_device.h"

namespace vr {

// two floats per packed VALU op (v_pk_add_f32 / v_pk_mul_f32 / v_pk_fma_f32 on gfx950)
typedef float f2 __attribute__((ext_vector_type(2)));

// ------------------------------------------------------------------------------------------------
// Ray / work-tile helpers
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ void ray_of_thread(const WorkTile& wt, int& x, int& y) {
    // lane -> y fastest so the 8 lanes of a row store 128 contiguous bytes of the x-major frame
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    x = wt.x0 + (wave & 1) * 8 + (lane >> 3);
    y = wt.y0 + (wave >> 1) * 8 + (lane & 7);
}

__device__ __forceinline__ int64_t out_index(int out_tiles, const WorkTile& wt, int x, int y, int H,
                                             int tile_w, int tile_h) {
    if (!out_tiles) return (int64_t)x * H + y;   // blendSampleColors: screen[x*H + y]
    const int tox = wt.tofs >> 16, toy = wt.tofs & 0xffff;
    const int i = tox + (x - wt.x0), j = toy + (y - wt.y0);
    return (int64_t)wt.slot * tile_w * tile_h + (int64_t)i * tile_h + j;
}

// Frame stores: the frame is written once and not re-read by the kernel, so the stores are
// non-temporal (no L2 allocation; the class volume keeps the cache).  Measured: C3 42.0 -> 40.1 us,
// a 1-sample frame 18.2 -> 15.7 us, tile assembly 9.4 -> 8.0 us.
__device__ __forceinline__ void store_f4(float4* p, float4 v) {
    __builtin_nontemporal_store(v.x, &p->x);
    __builtin_nontemporal_store(v.y, &p->y);
    __builtin_nontemporal_store(v.z, &p->z);
    __builtin_nontemporal_store(v.w, &p->w);
}

// A finished ray: float4 (r, g, b, 1) -- blendSampleColors sets alpha = 1 (kernel.cu:213) -- or,
// for VR_OUT_RGB tile buffers, the 3 colour floats only.
__device__ __forceinline__ void store_pixel(float4* out, int64_t idx, int rgb, float r, float g, float b) {
    if (rgb) {
        float* o = reinterpret_cast<float*>(out) + idx * 3;
        o[0] = r; o[1] = g; o[2] = b;
    } else {
        store_f4(out + idx, make_float4(r, g, b, 1.0f));
    }
}

// A raw buffer resource built from wave-uniform scalars at its point of use.  The march kernels
// hold ~100 SGPRs of frame constants; under that pressure the compiler once kept the resource of
// the general-view class gathers in VGPRs, and a resource operand in VGPRs gets a waterfall loop
// around EVERY load (4 readfirstlane + 2 compares + exec juggling per gather, found in the ISA).
// readfirstlane makes the operands provably uniform SGPRs again.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* base, int bytes) {
    const uint64_t p = (uint64_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)p);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
    const int n = __builtin_amdgcn_readfirstlane(bytes);
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), (short)0, n,
                                             0x00020000);
}

// Conservative [s_begin, s_end) of samples whose query point can lie in the box [lo, hi) (q units),
// for q(s) ~= base + s * step per axis.  Everything outside is guaranteed outside the box.  (Host
// too: TEST axis views take the march axis's range from the host, make_test.)
__host__ __device__ __forceinline__ void clip_range(const double base[3], const double step[3], const float lo[3],
                                           const float hi[3], int S, int& s_begin, int& s_end) {
    double a = 0.0, b = (double)(S - 1);
    for (int c = 0; c < 3; ++c) {
        if (fabs(step[c]) < 1e-30) {
            if (base[c] < (double)lo[c] || base[c] > (double)hi[c]) { s_begin = 0; s_end = 0; return; }
            continue;
        }
        double t0 = ((double)lo[c] - base[c]) / step[c], t1 = ((double)hi[c] - base[c]) / step[c];
        if (t0 > t1) { const double t = t0; t0 = t1; t1 = t; }
        a = fmax(a, t0); b = fmin(b, t1);
    }
    if (a > b) { s_begin = 0; s_end = 0; return; }
    const int sb = (int)floor(a) - 1, se = (int)ceil(b) + 2;
    s_begin = sb > 0 ? sb : 0;
    s_end = se < S ? se : S;
}

template <bool IDX64> struct IdxT { using type = int32_t; };
template <> struct IdxT<true> { using type = int64_t; };

__device__ __forceinline__ bool in_unit(float q) {
    // 0 <= q < 1  <=>  bits(q) < bits(1.0f) for every q except -0.0f, which q = p + 0.5f never is
    // (x + 0.5f == -0.0f is impossible in round-to-nearest); NaN is outside like the reference.
    return __float_as_uint(q) < 0x3f800000u;
}

// Counting passes (vr_count_work, never a timed launch): a lane's class gathers that touched memory,
// the bytes they read and the samples it evaluated, summed over the frame into stats[0], [2], [1]
__device__ __forceinline__ void count_work(unsigned long long* stats, unsigned gathers, unsigned bytes,
                                           unsigned samples) {
    if (gathers) atomicAdd(stats, (unsigned long long)gathers);
    if (samples) atomicAdd(stats + 1, (unsigned long long)samples);
    if (bytes) atomicAdd(stats + 2, (unsigned long long)bytes);
}

}  // namespace vr
