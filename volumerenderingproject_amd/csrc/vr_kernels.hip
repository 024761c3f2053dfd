// vr_kernels.hip -- hand-written gfx950 (CDNA4) kernels of the direct-volume ray marcher.
//
// Hot path: the reference materialises a W*H*S float4 sample
// buffer with one thread per (x, y, s) (calculateSampleColor kernel.cu:40-70 / getColorFromNF
// kernel.cu:72-187), then re-reads it per pixel (blendSampleColors kernel.cu:194-225).  Here ONE
// kernel marches each ray in registers: sample -> classify -> composite, O(1) memory per ray.
//
//   * VRC sampling (Octree::device_getIntensity, Octree.cu:286-311) is evaluated in closed form:
//     I(q) = max(0, R[floor(q * 2^D)]) inside [0,1)^3, where R is the octree's leaf grid.  The leaf
//     grid is separable -- leaf i on axis a maps to voxel map_a[i] or is outside the dataset
//     (Octree.cu:85-108) -- so three 2^D-entry int maps in LDS replace the 36-byte-node recursion.
//   * Classification (TransferFunction::getMaterial, TransferFunction.cu:46-55) depends only on
//     the voxel value, so it is done once per voxel into a uint8 class volume (exact); the march
//     reads 1 byte per sample and looks the colour up in an LDS table.
//   * Position arithmetic reproduces the reference's float op order (kernel.cu:53-59, glm mat4*vec4
//     type_mat4x4.inl:526-537) and is compiled with FP contraction off, so every leaf / voxel index
//     matches the reference exactly.
//   * Empty-space skipping uses a macro-cell occupancy bitmask over the leaf grid; a lane in an
//     empty cell jumps to the first sample that may leave the cell (conservative, so only alpha-0
//     samples are skipped: bitwise exact).  Early ray termination composites front to back.
//   * Workgroup = 16x16 rays (4 wave64s of 8x8); work tiles are dealt to XCDs in screen bands so
//     each XCD's L2 holds the slab of the class volume its rays touch.
// The TEST mode kernels are in vr_test.hip, the device helpers both use in vr_march.h.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <type_traits>

#include "vr_device.h"
#include "vr_march.h"

#pragma clang fp contract(off)

namespace vr {

// ------------------------------------------------------------------------------------------------
// Classification: per voxel class for VRC (octree value max(0,v) / (float)(int)cal_max, kernel.cu:64)
// and for TEST ((float)(v / cal_max) in double, kernel.cu:126).
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void classify_kernel(const float* __restrict__ vol, int64_t n,
                                                       float max_intensity, double cal_max,
                                                       const float* __restrict__ lo,
                                                       const float* __restrict__ hi, int n_tf,
                                                       uint8_t* __restrict__ cls_vrc,
                                                       uint8_t* __restrict__ cls_test,
                                                       const int64_t* __restrict__ lay, int64_t d2,
                                                       int64_t d3) {
    __shared__ float s_lo[kMaxTf], s_hi[kMaxTf];
    for (int i = threadIdx.x; i < n_tf; i += blockDim.x) { s_lo[i] = lo[i]; s_hi[i] = hi[i]; }
    __syncthreads();
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const float v = vol[i];
        // Octree.cu:303-305: res starts at 0 and takes a child value only if it is larger
        const float I = (v > 0.0f) ? v : 0.0f;
        if (cls_vrc) {
            // brick layout: offset = Fx[x] + Fy[y] + Fz[z] (separable, see OctreeHandler / vr_api.cpp)
            const int64_t x = i / (d2 * d3), y = (i / d3) % d2, z = i % d3;
            cls_vrc[lay[x] + lay[n / (d2 * d3) + y] + lay[n / (d2 * d3) + d2 + z]] =
                (uint8_t)tf_class(s_lo, s_hi, n_tf, I / max_intensity);
        }
        if (cls_test) cls_test[i] = (uint8_t)tf_class(s_lo, s_hi, n_tf, (float)((double)v / cal_max));
    }
}

// Packs the one-byte-per-slot classes into cbits-bit fields (cbits = 2 or 4): slot i at bit
// (i cbits) & 7 of byte (i cbits) >> 3 -- the march's bit addressing (VrcFrame.osh / omask).
__global__ __launch_bounds__(256) void pack_classes_kernel(const uint8_t* __restrict__ c8, int64_t slots, int cbits,
                                                           uint8_t* __restrict__ out) {
    const int per = 8 / cbits;
    const int64_t nbytes = (slots * cbits + 7) / 8;
    for (int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; b < nbytes; b += (int64_t)gridDim.x * blockDim.x) {
        unsigned v = 0;
        for (int j = 0; j < per; ++j) {
            const int64_t i = b * per + j;
            if (i < slots) v |= (unsigned)c8[i] << (j * cbits);
        }
        out[b] = (uint8_t)v;
    }
}

// ------------------------------------------------------------------------------------------------
// Occupancy of macro cells (2^cb leaves per axis) of the leaf grid.  A cell is occupied iff some
// leaf in it can produce a sample with alpha > 0.  maps: 3 x nleaf int (voxel index or -1).
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void occupancy_kernel(const uint8_t* __restrict__ cls,
                                                        const int32_t* __restrict__ maps, int nleaf,
                                                        int cb_shift, int ncell,
                                                        const int64_t* __restrict__ lx,
                                                        const int64_t* __restrict__ ly,
                                                        const int64_t* __restrict__ lz,
                                                        const uint8_t* __restrict__ alpha_nz,
                                                        int cls0, unsigned long long* __restrict__ occ) {
    const int64_t ncells = (int64_t)ncell * ncell * ncell;
    // grid-stride over blocks of 256 cells (single-leaf cells of a 2048^3 grid exceed one launch's
    // 2^32 threads); the stride keeps each wave on 64 consecutive cells, one bitmask word
    for (int64_t cell0 = (int64_t)blockIdx.x * blockDim.x; cell0 < ncells; cell0 += (int64_t)gridDim.x * blockDim.x) {
    const int64_t cell = cell0 + threadIdx.x;
    bool occupied = false;
    if (cell < ncells) {
        const int c[3] = {(int)(cell / ((int64_t)ncell * ncell)), (int)((cell / ncell) % ncell), (int)(cell % ncell)};
        int vmin[3], vmax[3];
        bool has_out = false, empty_axis = false;
        for (int a = 0; a < 3; ++a) {
            const int i0 = c[a] << cb_shift;
            const int i1 = min(nleaf, (c[a] + 1) << cb_shift);
            vmin[a] = 0x7fffffff; vmax[a] = -1;
            for (int i = i0; i < i1; ++i) {
                const int v = maps[a * nleaf + i];
                if (v < 0) { has_out = true; continue; }
                vmin[a] = min(vmin[a], v); vmax[a] = max(vmax[a], v);
            }
            if (vmax[a] < 0) empty_axis = true;
        }
        if (has_out && alpha_nz[cls0]) occupied = true;
        if (!occupied && !empty_axis) {
            for (int x = vmin[0]; x <= vmax[0] && !occupied; ++x)
                for (int y = vmin[1]; y <= vmax[1] && !occupied; ++y) {
                    const int64_t row = lx[x] + ly[y];
                    for (int z = vmin[2]; z <= vmax[2]; ++z)
                        if (alpha_nz[cls[row + lz[z]]]) { occupied = true; break; }
                }
        }
    }
    const unsigned long long m = __ballot(occupied);
    if ((threadIdx.x & 63) == 0 && cell < ncells) occ[cell >> 6] = m;
    }
}

// Column masks of the occupancy bitmask for axis-aligned views: for axis a and the two other cell
// coordinates (u, v) in increasing axis order, bit c of cols[a][u*ncell + v] = occupancy of the
// cell with coordinate c on axis a (ncell <= 64).
__global__ __launch_bounds__(256) void occ_columns_kernel(const unsigned long long* __restrict__ occ, int ncell,
                                                          unsigned long long* __restrict__ cols) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t per_axis = (int64_t)ncell * ncell;
    if (i >= 3 * per_axis) return;
    const int a = (int)(i / per_axis), u = (int)((i % per_axis) / ncell), v = (int)(i % ncell);
    unsigned long long m = 0;
    for (int c = 0; c < ncell; ++c) {
        const int cx = a == 0 ? c : u, cy = a == 0 ? u : (a == 1 ? c : v), cz = a == 2 ? c : v;
        const int64_t cell = ((int64_t)cx * ncell + cy) * ncell + cz;
        if ((occ[cell >> 6] >> (cell & 63)) & 1ull) m |= 1ull << c;
    }
    cols[i] = m;
}

// Column masks of one LEAF column each (axis-aligned views, nleaf <= kLeafColsMax): for axis a and
// the two other axes' leaf indices (u, v) in increasing axis order, bit c of cols[(a*nleaf + u)*nleaf
// + v] = some leaf of that column inside macro cell c along a is occupied (locc: the occupancy of
// single leaves, occupancy_kernel with cells of one leaf).  A ray of an axis view stays in its leaf
// column, so these masks are exact for it where the cell-column masks above are a 4x4-leaf superset.
__global__ __launch_bounds__(256) void leaf_columns_kernel(const unsigned long long* __restrict__ locc, int nleaf,
                                                           int cb_shift, unsigned long long* __restrict__ cols) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t per_axis = (int64_t)nleaf * nleaf;
    if (i >= 3 * per_axis) return;
    const int a = (int)(i / per_axis), u = (int)((i % per_axis) / nleaf), v = (int)(i % nleaf);
    unsigned long long m = 0;
    if (a == 2 && (nleaf & 63) == 0) {
        // along z a column's bits are consecutive: whole words, each covering 64 leaves (per-bit
        // loads here were one scattered 8-byte load per leaf and lane: 0.15 s at 2048^3)
        const unsigned long long* row = locc + (((int64_t)u * nleaf + v) * nleaf >> 6);
        const int per = cb_shift < 6 ? 64 >> cb_shift : 1;                 // cells per word
        const unsigned long long fmask = cb_shift < 6 ? (2ull << ((1 << cb_shift) - 1)) - 1ull : ~0ull;
        for (int k = 0; k < (nleaf >> 6); ++k) {
            const unsigned long long w = row[k];
            if (w == 0ull) continue;
            for (int j = 0; j < per; ++j)
                if ((w >> (j << min(cb_shift, 5))) & fmask) m |= 1ull << (((k << 6) >> cb_shift) + j);
        }
    } else {
        for (int l = 0; l < nleaf; ++l) {
            const int x = a == 0 ? l : u, y = a == 0 ? u : (a == 1 ? l : v), z = a == 2 ? l : v;
            const int64_t leaf = ((int64_t)x * nleaf + y) * nleaf + z;
            if ((locc[leaf >> 6] >> (leaf & 63)) & 1ull) m |= 1ull << (l >> cb_shift);
        }
    }
    cols[i] = m;
}

// Chebyshev distance (in cells, capped) from each macro cell to the nearest occupied one: every cell
// within max-norm distance dist - 1 of an empty cell is empty, so a ray may cross that whole box of
// cells in one jump.  One relaxation step per launch: d'(c) = occupied ? 0 : min(cap, 1 + min over
// the 26 neighbours of d); `cap` steps from d = (occupied ? 0 : cap) give the exact capped
// distance.  Cells beyond the grid count as empty: samples there are outside the cube, TF(0).
__global__ __launch_bounds__(256) void cell_dist_kernel(const unsigned long long* __restrict__ occ, int ncell,
                                                        const uint8_t* __restrict__ din, uint8_t* __restrict__ dout,
                                                        int cap, int init) {
    const int64_t n = (int64_t)ncell * ncell * ncell;
    const int64_t cell = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (cell >= n) return;
    if ((occ[cell >> 6] >> (cell & 63)) & 1ull) { dout[cell] = 0; return; }
    if (init) { dout[cell] = (uint8_t)cap; return; }
    const int cx = (int)(cell / ((int64_t)ncell * ncell)), cy = (int)((cell / ncell) % ncell), cz = (int)(cell % ncell);
    int m = cap;
    for (int dx = -1; dx <= 1; ++dx)
        for (int dy = -1; dy <= 1; ++dy)
            for (int dz = -1; dz <= 1; ++dz) {
                const int x = cx + dx, y = cy + dy, z = cz + dz;
                if ((dx | dy | dz) == 0 || x < 0 || y < 0 || z < 0 || x >= ncell || y >= ncell || z >= ncell) continue;
                m = min(m, (int)din[((int64_t)x * ncell + y) * ncell + z]);
            }
    dout[cell] = (uint8_t)min(cap, m + 1);
}

// ------------------------------------------------------------------------------------------------
// VRC march: fused calculateSampleColor + blendSampleColors (kernel.cu:40-70, :194-225).
// F2B = front to back with early termination (VR_FLAG_ERT); otherwise back to front exactly like
// the reference.  ESS = macro-cell empty-space skipping (VR_FLAG_ESS).  IDX64 = class volumes of
// 2^31 bytes or more.  AXIS1 = orthographic view along a volume axis (exactly one non-zero
// component of `front`, e.g. the reference's default camera and every axial / coronal / sagittal
// view): the two fixed coordinates of every sample are then bit-for-bit constant along the ray
// (P0 + t*0 = P0), so their leaf lookups are hoisted out of the march.  Every variant evaluates each
// sample with the reference's float op order; they differ only in what they can prove constant.
//
// Per lane the march evaluates samples in straight-line batches of K (K independent position /
// leaf / class-gather chains in flight), composites them in order, and -- with ESS -- jumps over
// macro cells that hold no alpha > 0 voxel before starting a batch.
// ------------------------------------------------------------------------------------------------
// Occupancy: forcing <= 80 SGPRs / 64 VGPRs (8 resident 256-thread workgroups per CU) made the
// K = 16 march spill and run 25-35 % slower on MI355X; the compiler's own allocation is kept,
// except for the axis-aligned ESS march with branch-free gathers at K = 16, where 7 waves/SIMD
// (72 VGPRs) measured 2 % faster than the compiler's 6 (C3, C2; round 1).
template <int GEOM, bool ESS, int K, bool SHADE>
#ifndef VR_RUNW_WAVES
#define VR_RUNW_WAVES 1
#endif
// (VR_GEN_WAVES: general-view ESS marches; 7 measured 1-3 % slower than the compiler's 6, round 6)
#ifndef VR_GEN_WAVES
#define VR_GEN_WAVES 1
#endif
constexpr int march_waves() {
    return GEOM == kGeomAxis1 && ESS && K == 16 && !SHADE ? 7
           : (GEOM == kGeomAxis1Run && ESS && !SHADE ? VR_RUNW_WAVES
                                                       : ((GEOM == kGeomOrtho || GEOM == kGeomConic) && ESS && !SHADE ? VR_GEN_WAVES : 1));
}
// (kGeomAxis1Run: uncapped -- its K = 16 form spills at 72 VGPRs)
// (An SGPR budget of 96 or 80 -- 7 / 8 resident workgroups per CU instead of the 6 that ~104 SGPRs
// allow -- measured 0-1 % on the default view and 2-5 % slower on general views: not kept.)
// premultiplied composites: TF reads issued kTfGroup at a time ahead of their composites (the
// default scheduling kept one LDS read in flight per sample); 8 or 16 spill at 72 VGPRs.  Same
// operations in the same order, so bitwise the same frames.  C3 -5 %, C2 -9 % (round 1 A/B)
constexpr int kTfGroup = 4;

// Per-ray geometry: q(s) = (org + t(s) * dir) + 0.5 with t(s) = s*sd + fc (modelAux =
// translate(0.5)).  Orthographic (kernel.cu:55-59): org = tlc + x*rsw/W*right + y*rsh/H*(-up), left
// to right, dir = front.  Conic (kernel.cu:30-34, :53-54; dead code in the reference, utils.h:28):
// dir = normalize(that point - cameraPos), org = cameraPos.  base ~ q(0) and stp = sd*dir serve the
// conservative clip of the sample range to the dataset box and the ESS jumps; samples outside the
// clip are TF(0) -- skipped when that is transparent.
template <bool CONIC>
__device__ __forceinline__ void ray_setup(const VrcFrame& f, int x, int y, float org[3], float dir[3], float base[3],
                                          float stp[3], float istp[3], int& s_begin, int& s_end) {
    const float A = (float)x * f.rsw / (float)f.W;
    const float B = (float)y * f.rsh / (float)f.H;
    float P0[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) P0[c] = (f.tlc[c] + A * f.right[c]) + B * (-f.up[c]);
    if (CONIC) {
        const float D[3] = {P0[0] - f.campos[0], P0[1] - f.campos[1], P0[2] - f.campos[2]};
        const float inv = 1.0f / sqrtf((D[0] * D[0] + D[1] * D[1]) + D[2] * D[2]);   // glm::normalize
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            org[c] = f.campos[c];
            dir[c] = D[c] * inv;
            stp[c] = f.sd * dir[c];
            istp[c] = stp[c] != 0.0f ? 1.0f / stp[c] : 0.0f;
        }
    } else {
#pragma unroll
        for (int c = 0; c < 3; ++c) { org[c] = P0[c]; dir[c] = f.front[c]; stp[c] = f.step[c]; istp[c] = f.inv_step[c]; }
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) base[c] = (org[c] + f.fc * dir[c]) + 0.5f;
    s_begin = 0;
    s_end = f.S;
    if (f.zero_transparent) {
        float a = 0.0f, bnd = (float)(f.S - 1);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            if (stp[c] == 0.0f) {
                if (base[c] < f.box_lo[c] || base[c] > f.box_hi[c]) { a = 1.0f; bnd = 0.0f; }
                continue;
            }
            const float t0 = (f.box_lo[c] - base[c]) * istp[c], t1 = (f.box_hi[c] - base[c]) * istp[c];
            a = fmaxf(a, fminf(t0, t1));
            bnd = fminf(bnd, fmaxf(t0, t1));
        }
        if (a > bnd) { s_end = 0; }
        else {
            s_begin = max(0, (int)floorf(a) - 1);
            s_end = min(f.S, (int)ceilf(bnd) + 2);
        }
    }
}

// Opt-in shading stage (VR_FLAG_SHADE; the north star's "Convolution central-difference gradient,
// LightInteraction Phong shading" -- the reference has neither on its render path: Convolution.cpp
// is an uncalled 10^3 toy stencil and LightInteraction.cpp returns 0).  Definition
// (restated bit for bit in oracle/vr_oracle.c or_shade):
//   g = ((v[x+1]-v[x-1]) * 0.5, (v[y+1]-v[y-1]) * 0.5, (v[z+1]-v[z-1]) * 0.5) over the raw float
//       volume at the sample's voxel, neighbour indices clamped to the volume;
//   headlight L = -front; N = -g / |g|; d = max(0, N.L); spec = ks * d^shininess (H = L);
//   rgb' = rgb * (ka + kd * d) + spec, alpha unchanged; |g| == 0 -> d = 1, spec = 0.
// Shading stage, per voxel: the outward unit normal of the central-difference gradient of the raw
// volume (one-sided at faces), N = -g/|g| with w = 1, or w = 0 where |g| = 0 -- the per-voxel part
// of VR_FLAG_SHADE, built once per volume (16 B per voxel) so a shaded sample costs one gather.
__global__ __launch_bounds__(256) void normal_kernel(const float* __restrict__ vol, int64_t d1, int64_t d2, int64_t d3,
                                                     float4* __restrict__ nrm) {
    const int64_t n = d1 * d2 * d3, sx = d2 * d3, sy = d3;
    for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < n; c += (int64_t)gridDim.x * blockDim.x) {
        const int64_t vx = c / sx, vy = (c / sy) % d2, vz = c % d3;
        const float gx = (vol[c + (vx + 1 < d1 ? sx : 0)] - vol[c - (vx > 0 ? sx : 0)]) * 0.5f;
        const float gy = (vol[c + (vy + 1 < d2 ? sy : 0)] - vol[c - (vy > 0 ? sy : 0)]) * 0.5f;
        const float gz = (vol[c + (vz + 1 < d3 ? 1 : 0)] - vol[c - (vz > 0 ? 1 : 0)]) * 0.5f;
        const float len2 = (gx * gx + gy * gy) + gz * gz;
        float4 o = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (len2 > 0.0f) {
            const float inv = 1.0f / sqrtf(len2);
            o = make_float4(-gx * inv, -gy * inv, -gz * inv, 1.0f);
        }
        nrm[c] = o;
    }
}

// Headlight Phong at a sample (oracle or_shade: same operations, same order):
// d = max(0, N.L), spec = ks * d^shininess, rgb' = rgb * (ka + kd d) + spec; flat (w = 0): d = 1.
__device__ __forceinline__ void shade_normal(const float4 nv, const float L[3], float ka, float kd, float ks,
                                             float shin, float& r, float& g, float& b) {
    float d = 1.0f, spec = 0.0f;
    if (nv.w != 0.0f) {
        const float ndl = (nv.x * L[0] + nv.y * L[1]) + nv.z * L[2];
        d = ndl > 0.0f ? ndl : 0.0f;
        // d^shininess as exp2(shininess * log2 d) on the hardware transcendentals (d > 0); d = 0 gives 0
        spec = d > 0.0f ? ks * __builtin_amdgcn_exp2f(shin * __builtin_amdgcn_logf(d)) : (shin == 0.0f ? ks : 0.0f);
    }
    const float k = ka + kd * d;
    r = r * k + spec;
    g = g * k + spec;
    b = b * k + spec;
}


// The class of a 32-bit class offset o (VrcFrame.osh / omask / cbits: bits below 8 bits per class,
// bytes at 8): the cbits-wide field at bit (o & omask) of byte o >> osh.  A negative o -- a table
// marker, kMapOut, an out-of-range select -- is an out-of-range byte offset: the load returns 0 and
// the field is class 0 without a memory access.
__device__ __forceinline__ int class_at(__amdgpu_buffer_rsrc_t rs, const VrcFrame& f, int o) {
    const int v = __builtin_amdgcn_raw_buffer_load_b8(rs, o >> f.osh, 0, 0);
    return (int)__builtin_amdgcn_ubfe((unsigned)v, (unsigned)(o & f.omask), (unsigned)f.cbits);
}

// The same for a valid (>= 0) 64-bit offset of an IDX64 class volume (a global load)
__device__ __forceinline__ int class_at64(const uint8_t* __restrict__ cls, const VrcFrame& f, int64_t o) {
    const unsigned v = cls[o >> f.osh];
    return (int)__builtin_amdgcn_ubfe(v, (unsigned)((int)o & f.omask), (unsigned)f.cbits);
}

// AXIS1 run words (VrcFrame.zrun; views along z).  A brick's z-run -- the classes of 8 consecutive
// z of one (x, y) -- is 8 * cbits bits inside one aligned 8-byte word, so the K samples of a batch
// (monotonic in z) lie in the words of its first and last samples whenever the batch spans at most
// two runs.  t = the sample's unit offset relative to its ray's word (off + zlow, VrcFrame.qsh / bsh);
// qa = t >> qsh of the first sample; (a0, a1) / (b0, b1) = the first / last sample's word.  The class
// of a sample in word a or b; run_miss says it is in neither (the caller then loads per sample).
__device__ __forceinline__ int run_class(const VrcFrame& f, int t, int qa, uint32_t a0, uint32_t a1, uint32_t b0,
                                         uint32_t b1) {
    const bool ina = (t >> f.qsh) == qa;
    const uint64_t w = ((uint64_t)(ina ? a1 : b1) << 32) | (ina ? a0 : b0);
    return (int)__builtin_amdgcn_ubfe((unsigned)(w >> ((unsigned)(t << f.bsh) & 63u)), 0u, (unsigned)f.cbits);
}
__device__ __forceinline__ bool run_miss(const VrcFrame& f, int t, int qa, int qb) {
    const int q = t >> f.qsh;
    return (q != qa) & (q != qb);
}

// AXIS1 table markers: far negative, so that fixed_off + marker is negative -- an out-of-range
// buffer offset -- for every class offset of a volume under 2^31 - 64 bytes (host: IDX64 above)
constexpr int32_t kTabTF0 = INT32_MIN + 1;    // TF(0): outside the unit cube or the dataset
constexpr int32_t kTabNone = INT32_MIN + 2;   // no sample: s outside [0, S)

// AXIS1 per-frame sample table (orthographic along volume axis ma, with right[ma] == up[ma] == 0,
// host-checked): the march-axis coordinate q(s) = (P0_ma + t(s) * front_ma) + 0.5 is the same for
// every ray of the frame, so its leaf lookup is a table over s: s_tab[s + K] = class-offset
// contribution of axis ma (>= 0), kTabTF0 (outside the cube or dataset) or kTabNone (s outside
// [0, S)).  The same float expressions as the per-ray statement, so every index is unchanged.  For
// ESS, s_cel = the macro cell of q(s) along ma (-1 below the cube, ncell above) -- monotonic in s --
// and s_entry[c] = the first sample in march order whose cell is c or beyond it in the direction of
// travel (F2B: S if none; B2F: -1 if none): a jump to the next occupied cell of the ray's column is
// one LDS read, exact, with no safety margin.  Ends with the table complete in LDS (barrier).
// SPLIT (views along z, kGeomAxis1Z): an entry is int2 {byte offset, bit} of the contribution -- the
// fixed (x, y) part of a ray's class offset is then byte-aligned (host), so a gather is one add and
// one v_bfe_u32, no shift / mask per sample; markers keep their value in .x (bit 0).
template <bool F2B, bool ESS, int K, typename TabE>
__device__ __forceinline__ void axis1_table(const VrcFrame& f, int ma, bool cells_up, const int32_t* s_map,
                                            TabE* s_tab, int8_t* s_cel, int32_t* s_entry) {
    const int n_tab = f.S + 2 * K;
    const float P0m = (f.tlc[ma] + 0.0f * f.right[ma]) + 0.0f * (-f.up[ma]);
    const float front_m = f.front[ma];
    for (int j = threadIdx.x; j < n_tab; j += kWgThreads) {
        const int s = j - K;
        int m = kTabNone, cel = 0;
        if (s >= 0 && s < f.S) {
            const float t = (float)s * f.sd + f.fc;
            const float q = (P0m + t * front_m) + 0.5f;   // modelAux = translate(0.5)
            if (in_unit(q)) {
                const int i = (int)(q * f.leaves);
                const int mm = s_map[i];
                m = mm >= 0 ? mm : kTabTF0;
                cel = i >> f.cb_shift;
            } else {
                m = kTabTF0;
                cel = q < 0.0f ? -1 : f.ncell;
            }
        }
        if constexpr (sizeof(TabE) == 8) s_tab[j] = m >= 0 ? make_int2(m >> f.osh, m & f.omask) : make_int2(m, 0);
        else s_tab[j] = m;
        if (ESS) s_cel[j] = (int8_t)cel;
    }
    __syncthreads();
    if (ESS) {
        for (int c = threadIdx.x; c < f.ncell; c += kWgThreads) {
            // predicate "cell(s) is c or beyond": monotone in s (F2B false..true, B2F true..false)
            auto beyond = [&](int s) { const int v = s_cel[s + K]; return cells_up ? v >= c : v <= c; };
            int lo = 0, hi = f.S;   // F2B: first s with beyond; B2F: last s with beyond (lo - 1)
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (F2B ? beyond(mid) : !beyond(mid)) hi = mid; else lo = mid + 1;
            }
            s_entry[c] = F2B ? lo : lo - 1;
        }
        __syncthreads();
    }
}

template <bool F2B, bool ESS, bool IDX64, int GEOM, int K, bool SHADE, int STATS = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(march_waves<GEOM, ESS, K, SHADE>()))) void vrc_march_kernel(VrcFrame f, const WorkTile* __restrict__ work,
                                                        const int32_t* __restrict__ order,
                                                        const uint8_t* __restrict__ cls,
                                                        const int32_t* __restrict__ gmaps,
                                                        const int64_t* __restrict__ gmapx64,
                                                        const uint32_t* __restrict__ gocc,
                                                        const float4* __restrict__ tf_rgba, int n_tf,
                                                        float4* __restrict__ out,
                                                        unsigned long long* __restrict__ stats,
                                                        const float* __restrict__ vol,
                                                        const int32_t* __restrict__ rawmaps,
                                                        const unsigned long long* __restrict__ occcol,
                                                        const uint8_t* __restrict__ cdist,
                                                        const int32_t* __restrict__ gtab,
                                                        int32_t* __restrict__ gtab_out) {
    using idx_t = typename IdxT<IDX64>::type;
    constexpr bool AXIS1 = GEOM == kGeomAxis1 || GEOM == kGeomAxis1Run || GEOM == kGeomAxis1Z;
    constexpr bool CONIC = GEOM == kGeomConic;
    constexpr bool RUNW = GEOM == kGeomAxis1Run;   // run-word class gathers (host: f.zrun)
    constexpr bool SPLIT = GEOM == kGeomAxis1Z;     // split {byte, bit} view table (host: f.tsplit)
    using TabE = typename std::conditional<SPLIT, int2, int32_t>::type;
    constexpr int kTabWords = SPLIT ? 2 : 1;
    unsigned long long t_entry = 0;
    if (STATS == 1) t_entry = __builtin_amdgcn_s_memrealtime();
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    // LDS: [tf rgba (n_tf + 1) x 16 B; entry n_tf = (0,0,0,0), "no sample"]
    //      general views: [x map idx_t x nleaf][y, z maps int32 2 x nleaf]
    //      AXIS1: [march-axis map int32 x nleaf]
    //      [SHADE: raw leaf -> voxel maps 3 x nleaf]
    //      AXIS1: [sample table int32 x (S + 2K)][ESS: entry int32 x ncell][ESS: cell int8 x (S + 2K)]
    // First round of loads: the first slot's work tile, the TF entries and the staging loads below
    // are all issued before any branch on a kernel argument -- guarded loads would make the compiler
    // load each argument under the branch that needs it, a chain of dependent scalar round trips
    // (six before the first vector load in the round-4 ISA of the default-view march).  The work
    // tile load is unconditional (index clamped; a background-only workgroup leaves before using it).
    // (`order`, a block -> work-entry indirection, is unused: every caller passes null, and testing
    // it put one more dependent scalar round trip in front of the first load)
    const int b_first = (int)blockIdx.x;
    const bool b_ok = b_first >= 0 && b_first < f.n_work;
    WorkTile wt_first = work[b_ok ? b_first : 0];
    if (!b_ok) wt_first = WorkTile{0, 0, 0, 0};
    // the frame constants the exits below branch on, loaded in the first round: left to the
    // compiler, each is loaded (and waited for) inside the branch that first needs it
    asm volatile("" ::"s"(f.out_tiles), "s"(f.bg_first), "s"(f.n_slots), "s"(f.n_hull), "s"(f.W), "s"(f.H),
                 "s"((uint64_t)gtab_out), "s"((uint64_t)tf_rgba));
    const int ma = AXIS1 ? f.axis1 : 0;
    float4* s_tf = reinterpret_cast<float4*>(smem);
    unsigned char* p = smem + (size_t)(n_tf + 1) * sizeof(float4);
    // general views: each leaf map has f.pad kMapOut entries on either side (s_mx[-pad .. nleaf + pad))
    const int pad = AXIS1 ? 0 : f.pad;
    idx_t* s_mx = reinterpret_cast<idx_t*>(p) + pad;
    int32_t* s_my = nullptr;
    int32_t* s_mz = nullptr;
    int32_t* s_map = reinterpret_cast<int32_t*>(p);   // AXIS1: map of the march axis
    if (!AXIS1) {
        const int span = f.nleaf + 2 * pad;
        p += (size_t)span * sizeof(idx_t);
        s_my = reinterpret_cast<int32_t*>(p) + pad;
        s_mz = s_my + span;
        p += (size_t)2 * span * sizeof(int32_t);
    } else {
        p += (size_t)f.nleaf * sizeof(int32_t);
    }
    // ESS state lives outside LDS: AXIS1 keeps per-ray column masks in registers (occcol), other
    // views read the cell-distance field (cdist, L1/L2 resident)
    int32_t* s_raw = reinterpret_cast<int32_t*>(p);
    if (SHADE) p += (size_t)3 * f.nleaf * sizeof(int32_t);
    const int n_tab = f.S + 2 * K;
    TabE* s_tab = reinterpret_cast<TabE*>(p);
    int32_t* s_entry = reinterpret_cast<int32_t*>(s_tab + n_tab);
    int8_t* s_cel = reinterpret_cast<int8_t*>(s_entry + f.ncell);
    // class gathers through a buffer resource (raw, bound = class bytes; unused for IDX64 volumes)
    const __amdgpu_buffer_rsrc_t crs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(cls), (short)0, IDX64 ? 0 : f.cls_bytes, 0x00020000);
    // staging loads first (independent of the work tile), then the culled-tile exit
    // AXIS1: the view table (tab | entry | cel) a previous launch of the same view published, or the
    // march-axis map to build it from.  The first round of staging loads is issued before the
    // culled-tile test and written to LDS after it, so a culled tile (e.g. one over empty cell
    // columns, frame_list) waits for its work-tile load only.
    // (workgroup 0 of a publishing launch builds the view table even when its own tile is culled)
    const bool publish = AXIS1 && gtab_out != nullptr && blockIdx.x == 0;
    auto culled_exit = [&]() -> bool {
        // (bitwise &: every operand is evaluated, no short-circuit chain of scalar loads and branches)
        if ((f.out_tiles == 0) & (wt_first.slot < 0) & ((int)gridDim.x >= f.n_slots) & !publish) {
            // a culled whole-frame tile: exactly the background
            int x, y;
            ray_of_thread(wt_first, x, y);
            if (x < f.W && y < f.H) store_f4(out + (int64_t)x * f.H + y, make_float4(f.bg[0], f.bg[1], f.bg[2], 1.0f));
            return true;
        }
        return false;
    };
    // Per-ray state.  AXIS1: the two fixed axes a0 < a1 are hoisted (q_c = P0_c + 0.5 exactly since
    // front_c == 0; t * 0 adds a signed zero), their leaf -> class-offset maps read from global (L2
    // resident) together with the ray's occupancy column, all in one round of loads.
    struct Ray {
        int x, y, s_begin, s_end;
        float P0[3], dir[3], base[3], stp[3], istp[3];   // P0 = the ray origin (org)
        idx_t fixed_off;
        bool fixed_in;
        unsigned long long colmask;   // AXIS1 + ESS: occupancy of the ray's cell column, bit = cell on axis ma
    };
    auto init_ray = [&](const WorkTile& wt, Ray& R) {
        ray_of_thread(wt, R.x, R.y);
        ray_setup<CONIC>(f, R.x, R.y, R.P0, R.dir, R.base, R.stp, R.istp, R.s_begin, R.s_end);
        R.fixed_off = 0;
        R.fixed_in = true;
        R.colmask = 0;
        if (AXIS1) {
            const int a0 = ma == 0 ? 1 : 0, a1 = ma == 2 ? 1 : 2;
            const float q0 = (ma == 0 ? R.P0[1] : R.P0[0]) + 0.5f;
            const float q1 = (ma == 2 ? R.P0[1] : R.P0[2]) + 0.5f;
            // leaf indices clamped so the lookups are unconditional (an out-of-cube axis makes the
            // whole ray TF(0) anyway)
            const unsigned lim = (unsigned)(f.nleaf - 1);
            const int i0 = (int)min((unsigned)(int)(q0 * f.leaves), lim);
            const int i1 = (int)min((unsigned)(int)(q1 * f.leaves), lim);
            const idx_t m0 = (IDX64 && a0 == 0) ? (idx_t)gmapx64[i0] : (idx_t)gmaps[a0 * f.nleaf + i0];
            const idx_t m1 = (idx_t)gmaps[a1 * f.nleaf + i1];
            // (f.leafcols: occcol holds one mask per leaf column, leaf_columns_kernel)
            if (ESS)
                R.colmask = occcol[f.leafcols ? ((size_t)ma * f.nleaf + i0) * f.nleaf + i1
                                              : ((size_t)ma * f.ncell + (i0 >> f.cb_shift)) * f.ncell + (i1 >> f.cb_shift)];
            R.fixed_in = ((int)in_unit(q0) & (int)in_unit(q1) & (int)(m0 >= 0) & (int)(m1 >= 0)) != 0;
            R.fixed_off = m0 + m1;
            if (!R.fixed_in && f.zero_transparent) R.s_end = 0;   // the whole ray is TF(0)
            // ESS: a column without an occupied cell holds only alpha-0 samples (exact no-ops of either
            // blend): no batch at all, instead of one batch of no-ops after the first empty-cell jump
            if (ESS && R.colmask == 0ull && f.zero_transparent) R.s_end = 0;
        }
    };
    Ray R;
    // the TF entries join the first round of staging loads (n_tf <= kMaxTf = kWgThreads, host)
    // (unconditional, index clamped: the staging loop below stores it only for threadIdx.x < n_tf)
    const float4 tfc = tf_rgba[(int)threadIdx.x < n_tf ? (int)threadIdx.x : 0];
    // general views, 32-bit offsets: the three padded leaf maps (contiguous in LDS from s_mx - pad,
    // kMapOut outside the dataset and in the padding) join the first round as well
    const int gspan = f.nleaf + 2 * pad, gn = (AXIS1 || IDX64) ? 0 : 3 * gspan;
    // entry i of the padded maps.  For these launches gmaps is the host's copy with kMapPadMax kMapOut
    // entries either side of each axis (pmaps_pad), so entry i of axis a = i / gspan sits at
    // i + (2a + 1)(kMapPadMax - pad): one buffer load, no range test or select.  (The loads are
    // unconditional: under a range test the compiler waited for each inside its branch, eight L2
    // round trips in series before the staging barrier -- the round-4 ISA.  Past 3 gspan the offset
    // may leave the buffer: it reads 0, which is never stored.)
    const int gpd = kMapPadMax - pad;
    const __amdgpu_buffer_rsrc_t gmr = uniform_rsrc(gmaps, 3 * (f.nleaf + 2 * kMapPadMax) * 4);
    auto gmap_entry = [&](int i) -> int32_t {
        const int a = (int)(i >= gspan) + (int)(i >= 2 * gspan);
        return (int32_t)__builtin_amdgcn_raw_buffer_load_b32(gmr, (i + (2 * a + 1) * gpd) * 4, 0, 0);
    };
    // 16 B per load when no int4 straddles two axes (gspan a multiple of 4: the host rounds pad up to
    // a multiple of 4, and nleaf is a power of two), as for the axis views' table
    const bool g4 = (gspan & 3) == 0;
    int4 gq[2];
    int32_t gv[8];
    if (!AXIS1 && !IDX64) {
        if (g4) {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int i = ((int)threadIdx.x + u * kWgThreads) * 4;
                const int a = (int)(i >= gspan) + (int)(i >= 2 * gspan);
                const auto w = __builtin_amdgcn_raw_buffer_load_b128(gmr, (i + (2 * a + 1) * gpd) * 4, 0, 0);
                gq[u] = make_int4((int)w[0], (int)w[1], (int)w[2], (int)w[3]);
            }
        } else {
#pragma unroll
            for (int u = 0; u < 8; ++u) gv[u] = gmap_entry((int)threadIdx.x + u * kWgThreads);
        }
    }
    // Lockstep (round 6): views along z with the split table, front to back, premultiplied, ESS --
    // the C3 / C4 default camera.  See the march loop below.
#ifndef VR_VRC_LOCK
#define VR_VRC_LOCK 0
#endif
    constexpr bool LOCKV = VR_VRC_LOCK && SPLIT && !IDX64 && F2B && !SHADE && ESS && STATS != 1;
    // (the wave reads the published view table through scalar loads: no LDS copy of it)
    const bool lock_run = LOCKV && f.zero_transparent && f.cls0 == 0;
    const bool lock_scalar = lock_run && gtab != nullptr;
    // AXIS1: the view table's (or the march-axis map's) first round of staging loads
    int32_t* dst = gtab ? reinterpret_cast<int32_t*>(s_tab) : s_map;
    const int32_t* src = gtab ? gtab : gmaps + (size_t)ma * f.nleaf;   // int32 for every AXIS1 launch (host)
    const int n = gtab ? (n_tab * 4 * kTabWords + f.ncell * 4 + n_tab + 3) / 4 : f.nleaf;
    // 16 B per thread per load (2 x 256 x 16 B = 8 KB in the first round; the C3 default view's table
    // is ~5 KB): a quarter of the load and LDS-store instructions of 4-B staging.  Whole int4s: the
    // host pads the published table's buffer and the LDS carve-up by 16 B (vrc_lds_bytes), and the
    // march-axis map is nleaf (a multiple of 4) entries
    const int n4 = (n + 3) >> 2;
    int4 v4[2];
    if (AXIS1 && !lock_scalar) {
        const __amdgpu_buffer_rsrc_t srs = uniform_rsrc(src, n4 * 16);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int i = (int)threadIdx.x + u * kWgThreads;   // (past n4: out of range, reads 0)
            const auto w = __builtin_amdgcn_raw_buffer_load_b128(srs, i * 16, 0, 0);
            v4[u] = make_int4((int)w[0], (int)w[1], (int)w[2], (int)w[3]);
        }
    }
    if ((f.out_tiles == 0) & ((int)blockIdx.x >= f.bg_first)) {
        // a background-only workgroup: bg_group culled work tiles off the projected dataset box,
        // each exactly the background (no staging, no march)
        const int e0 = f.bg_first + ((int)blockIdx.x - f.bg_first) * f.bg_group;
        for (int i = 0; i < f.bg_group; ++i) {
            const int e = e0 + i;
            if (e >= f.n_work) break;
            int x, y;
            ray_of_thread(work[e], x, y);
            if (x < f.W && y < f.H) store_f4(out + (int64_t)x * f.H + y, make_float4(f.bg[0], f.bg[1], f.bg[2], 1.0f));
        }
        return;
    }
    if (!AXIS1 && ((f.n_hull > 0) & (f.out_tiles == 0) & ((int)gridDim.x >= f.n_slots) & (wt_first.slot >= 0) & b_ok)) {
        // general views: a work tile inside the visible rectangle but off the projected box's hull
        // (separated by one of its edges) sees only TF(0) / empty cells -- exactly the background,
        // like the rectangle's culled tiles -- so it exits before the staging stores.  Wave-uniform:
        // the tile's pixels [x0, x0 + 16) x [y0, y0 + 16) against each edge's half-plane.
        const float x0 = (float)wt_first.x0, y0 = (float)wt_first.y0;
        bool off = false;
        // unrolled over kMaxHull: the edges' kernel-argument loads issue together, not one
        // dependent scalar round trip per loop iteration
#pragma unroll
        for (int e = 0; e < kMaxHull; ++e) {
            const float nx = f.hull[e][0], ny = f.hull[e][1];
            const float px = nx > 0.0f ? x0 : x0 + (float)(kWgRaysX - 1);
            const float py = ny > 0.0f ? y0 : y0 + (float)(kWgRaysY - 1);
            off |= (e < f.n_hull) & (nx * px + ny * py > f.hull[e][2]);   // (bitwise: no branch per edge)
        }
        if (off) {
            int x, y;
            ray_of_thread(wt_first, x, y);
            if (x < f.W && y < f.H) store_f4(out + (int64_t)x * f.H + y, make_float4(f.bg[0], f.bg[1], f.bg[2], 1.0f));
            return;
        }
    }
    if (AXIS1) {
        if (culled_exit()) return;
        init_ray(wt_first, R);   // the ray's map / column loads: issued before the staging stores wait
        if (!lock_scalar) {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int i = (int)threadIdx.x + u * kWgThreads;
                if (i < n4) reinterpret_cast<int4*>(dst)[i] = v4[u];
            }
            // the rest (long rays, e.g. C4's S = 1024 table of ~10 KB) in int4s as well
            for (int i = (int)threadIdx.x + 2 * kWgThreads; i < n4; i += kWgThreads)
                reinterpret_cast<int4*>(dst)[i] = reinterpret_cast<const int4*>(src)[i];
        }
    }
    // front-to-back without shading composites premultiplied entries (a*r, a*g, a*b, 1 - a):
    // C += T * (a*c), T *= (1 - a) -- two fewer operations per sample than w = T*a, C += w*c; the
    // reassociation is of the kind ERT already allows, and alpha 0 stays an exact no-op
    constexpr bool PREMUL = F2B && !SHADE;
    // the LDS table holds (a*r, a*g, a*b, 1 - a) whenever the colour is not shaded per sample: the
    // back-to-front blend r' = r*(1 - a) + c*a is then r' = r*e.w + e.x with the same two products
    // rounded once per entry instead of per sample -- bitwise the reference's expression
    constexpr bool PTAB = !SHADE;
    for (int i = threadIdx.x; i <= n_tf; i += kWgThreads) {
        float4 c = i < n_tf ? tfc : make_float4(0.0f, 0.0f, 0.0f, 0.0f);   // (i < n_tf: i is this thread's)
        if (PTAB) c = make_float4(c.x * c.w, c.y * c.w, c.z * c.w, 1.0f - c.w);
        s_tf[i] = c;
    }
    if (!AXIS1 && culled_exit()) return;
    if (!AXIS1) init_ray(wt_first, R);
    if (!AXIS1 && !IDX64) {
        int32_t* gbase = reinterpret_cast<int32_t*>(s_mx) - pad;
        if (g4) {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int i4 = (int)threadIdx.x + u * kWgThreads;
                if (i4 * 4 < gn) reinterpret_cast<int4*>(gbase)[i4] = gq[u];
            }
        } else {
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int i = (int)threadIdx.x + u * kWgThreads;
                if (i < gn) gbase[i] = gv[u];
            }
        }
        for (int i = (int)threadIdx.x + 8 * kWgThreads; i < gn; i += kWgThreads) gbase[i] = gmap_entry(i);
    } else if (!AXIS1)
        for (int i = (int)threadIdx.x - pad; i < f.nleaf + pad; i += kWgThreads) {
            const bool in = (unsigned)i < (unsigned)f.nleaf;   // padding: outside the unit cube
            if (IDX64) s_mx[i] = in ? (idx_t)gmapx64[i] : (idx_t)kMapOut;
            else s_mx[i] = (idx_t)(!in || gmaps[i] < 0 ? kMapOut : gmaps[i]);
            s_my[i] = !in || gmaps[f.nleaf + i] < 0 ? kMapOut : gmaps[f.nleaf + i];
            s_mz[i] = !in || gmaps[2 * f.nleaf + i] < 0 ? kMapOut : gmaps[2 * f.nleaf + i];
        }
    if (SHADE)
        for (int i = threadIdx.x; i < 3 * f.nleaf; i += kWgThreads) s_raw[i] = rawmaps[i];

    __syncthreads();
    unsigned long long t_b1 = 0, t_b2 = 0;
    if (STATS == 1) t_b1 = __builtin_amdgcn_s_memrealtime();

    // AXIS1 (orthographic along volume axis ma, with right[ma] == up[ma] == 0, host-checked): the
    // march-axis coordinate q(s) = (P0_ma + t(s) * front_ma) + 0.5 is the same for every ray of the
    // frame, so its leaf lookup is a per-frame table over s: s_tab[s + K] = class-offset contribution
    // of axis ma (>= 0), -1 = TF(0) (outside the cube or dataset), -2 = no sample (s outside [0, S)).
    // The same float expressions as the per-ray statement, so every index is unchanged.  For ESS,
    // s_cel = the macro cell of q(s) along ma (-1 below the cube, ncell above) -- monotonic in s --
    // and s_entry[c] = the first sample in march order whose cell is c or beyond it in the
    // direction of travel (F2B: S if none; B2F: -1 if none): a jump to the next occupied cell of
    // the ray's column is one LDS read, exact, with no safety margin.
    const bool cells_up = F2B ? (f.step[ma] > 0.0f) : (f.step[ma] < 0.0f);   // cell index grows in march order
    if (AXIS1) {
        if (!gtab) {
            axis1_table<F2B, ESS, K, TabE>(f, ma, cells_up, s_map, s_tab, s_cel, s_entry);
            if (publish)   // the view's table for the launches after this one (same stream, so ordered)
                for (int i = threadIdx.x; i < (n_tab * 4 * kTabWords + f.ncell * 4 + n_tab + 3) / 4; i += kWgThreads)
                    gtab_out[i] = reinterpret_cast<const int32_t*>(s_tab)[i];
        }   // else: staged from the previous launch's copy with the first round of loads
        if (STATS == 1) t_b2 = __builtin_amdgcn_s_memrealtime();
    }
    const float Lh[3] = {-f.front[0], -f.front[1], -f.front[2]};   // headlight (SHADE)

    // Persistent when gridDim < n_slots: a workgroup walks slots blockIdx.x, +gridDim.x, ... (gridDim
    // is a multiple of 8, so a workgroup stays on the XCD band its first slot belongs to).
    for (int blk = blockIdx.x; blk < f.n_slots; blk += gridDim.x) {
    unsigned long long t_start = 0;
    if (STATS == 1) t_start = __builtin_amdgcn_s_memrealtime();
    const bool first = blk == (int)blockIdx.x;
    const int b = first ? b_first : blk;
    if (b < 0 || b >= f.n_work) continue;
    const WorkTile wt = first ? wt_first : work[b];
    if (!first) init_ray(wt, R);
    const int x = R.x, y = R.y;
    const bool lane_ok = x < f.W && y < f.H;
    if (!lock_run && !lane_ok) continue;   // (lockstep: every lane takes part in the wave's reductions)
    if (!f.out_tiles && wt.slot < 0) {   // culled tile (persistent grids reach them here)
        if (lane_ok) store_f4(out + (int64_t)x * f.H + y, make_float4(f.bg[0], f.bg[1], f.bg[2], 1.0f));
        continue;
    }
    unsigned st_iter = 0, st_jumps = 0, st_loads = 0, st_bytes = 0;
    const float* P0 = R.P0;
    const float* dir = R.dir;
    const float* base = R.base;
    const float* stp = R.stp;
    const float* istp = R.istp;
    const int s_begin = R.s_begin, s_end = R.s_end;
    const idx_t fixed_off = R.fixed_off;
    const bool fixed_in = R.fixed_in;
    const int zlow = (int)fixed_off & ((1 << f.qsh) - 1);   // run words: fixed_off's offset in its word
    const int notin = fixed_in ? 0 : INT32_MIN;   // AXIS1: makes every table entry invalid for a ray off the dataset
    const unsigned long long colmask = R.colmask;

    float r, g, bl;      // F2B: accumulated colour; B2F: fragment colour
    float T = 1.0f;
    if (F2B) { r = 0.0f; g = 0.0f; bl = 0.0f; }
    else { r = f.bg[0]; g = f.bg[1]; bl = f.bg[2]; }

    // class offset of sample s (general views): >= 0 voxel class offset, -1 = TF(0) (outside cube or dataset)
    auto sample_off = [&](int s, int& cell, int (&cc)[3]) -> idx_t {
        const float t = (float)s * f.sd + f.fc;
        {
            const float qx = (P0[0] + t * dir[0]) + 0.5f;
            const float qy = (P0[1] + t * dir[1]) + 0.5f;
            const float qz = (P0[2] + t * dir[2]) + 0.5f;
            const unsigned lim = (unsigned)(f.nleaf - 1);
            const unsigned ix = min((unsigned)(int)(qx * f.leaves), lim);
            const unsigned iy = min((unsigned)(int)(qy * f.leaves), lim);
            const unsigned iz = min((unsigned)(int)(qz * f.leaves), lim);
            cc[0] = (int)(ix >> f.cb_shift); cc[1] = (int)(iy >> f.cb_shift); cc[2] = (int)(iz >> f.cb_shift);
            cell = __mul24(__mul24(cc[0], f.ncell) + cc[1], f.ncell) + cc[2];   // (< 64^3)
            const idx_t mx = s_mx[ix];
            const int32_t my = s_my[iy], mz = s_mz[iz];
            const bool ok = in_unit(qx) && in_unit(qy) && in_unit(qz) && (mx | (idx_t)my | (idx_t)mz) >= 0;
            return ok ? mx + (idx_t)my + (idx_t)mz : (idx_t)-1;
        }
    };

    // macro cell of sample s (ESS, general views); false if the sample lies outside the unit cube
    auto sample_cell = [&](int s, int& cell, int (&cc)[3]) -> bool {
        const float t = (float)s * f.sd + f.fc;
        {
            const float qx = (P0[0] + t * dir[0]) + 0.5f;
            const float qy = (P0[1] + t * dir[1]) + 0.5f;
            const float qz = (P0[2] + t * dir[2]) + 0.5f;
            const unsigned lim = (unsigned)(f.nleaf - 1);
            const unsigned ix = min((unsigned)(int)(qx * f.leaves), lim);
            const unsigned iy = min((unsigned)(int)(qy * f.leaves), lim);
            const unsigned iz = min((unsigned)(int)(qz * f.leaves), lim);
            cc[0] = (int)(ix >> f.cb_shift); cc[1] = (int)(iy >> f.cb_shift); cc[2] = (int)(iz >> f.cb_shift);
            cell = __mul24(__mul24(cc[0], f.ncell) + cc[1], f.ncell) + cc[2];   // (< 64^3)
            return in_unit(qx) && in_unit(qy) && in_unit(qz);
        }
    };

    if constexpr (LOCKV) {
    if (lock_run) {
        // Lockstep march of the wave.  Every ray of an axis view shares the march axis's sample
        // sequence and clip range, and only its own empty-cell jumps (leaf-column masks) made the lanes
        // drift apart.  Here the wave marches one sequence: the view-table entries, cells and cell
        // entries are wave-uniform -- scalar loads from the published copy (gtab; the prologue staged
        // nothing) or broadcast LDS reads moved to scalar registers (the publishing launch) -- and the
        // empty-cell jumps follow the union of the wave's masks.  A lane in one of its own empty cells
        // gathers classes of alpha 0 and composites exact no-ops; a lane off the dataset or the frame
        // gathers out of range (class 0, the premultiplied (0, 0, 0, 1)): exact no-ops too.  Lanes go
        // on compositing after their own T < eps until the whole wave is there: what they add is below
        // eps (front to back, within the ERT tolerance).
        const bool act = lane_ok && s_begin < s_end;   // (init_ray: s_end = 0 off the dataset / empty column)
        unsigned long long wm = act ? colmask : 0ull;
        int wsb = act ? s_begin : INT32_MAX, wse = act ? s_end : INT32_MIN;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            wm |= __shfl_xor(wm, o);
            wsb = min(wsb, __shfl_xor(wsb, o));
            wse = max(wse, __shfl_xor(wse, o));
        }
        wsb = __builtin_amdgcn_readfirstlane(wsb);
        wse = __builtin_amdgcn_readfirstlane(wse);
        wm = ((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(wm >> 32)) << 32) |
             (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)wm);
        const int fixedB = act ? (int)(fixed_off >> f.osh) : (INT32_MIN / 2);
        const int n_tab_l = f.S + 2 * K;
        // the published copy through the constant address space: wave-uniform addresses there compile to
        // scalar loads (s_load) into SGPRs -- the scalar cache serves every wave of the frame
        typedef const __attribute__((address_space(4))) int32_t cint;
        cint* gtw = (cint*)gtab;
        cint* gent = gtw + 2 * n_tab_l;   // (published: tab | entry | cel, int32 words)
        cint* gcelw = gent + f.ncell;
        typedef const volatile __attribute__((address_space(3))) unsigned long long lds_u64;
        float ert_eps_l = f.ert_eps;
        asm volatile("" : "+v"(ert_eps_l));
        // one copy of the loop per source of the table (scalar loads from the published copy, or the
        // LDS copy of a publishing launch), so no per-entry branch stands between the scalar loads
        auto lock_march = [&](auto sc_tag) {
            constexpr bool SC = decltype(sc_tag)::value;
            // (readfirstlane: the LDS values are wave-uniform; it makes them scalar registers)
            auto tab_at = [&](int j) -> int2 {
                if constexpr (SC) return make_int2(gtw[2 * j], gtw[2 * j + 1]);
                const unsigned long long u = ((lds_u64*)(s_tab))[j];
                return make_int2(__builtin_amdgcn_readfirstlane((int)(uint32_t)u),
                                 __builtin_amdgcn_readfirstlane((int)(uint32_t)(u >> 32)));
            };
            auto cel_at = [&](int j) -> int {
                if constexpr (SC) {   // (bytes from a scalar dword: no scalar byte loads on gfx950)
                    const int wv = gcelw[j >> 2];
                    return (int)(int8_t)(wv >> (8 * (j & 3)));
                }
                return __builtin_amdgcn_readfirstlane((int)s_cel[j]);
            };
            auto entry_at = [&](int c) -> int {
                if constexpr (SC) return gent[c];
                return __builtin_amdgcn_readfirstlane(s_entry[c]);
            };
            int su = wsb;
            bool wdone = wsb >= wse;
            while (!wdone) {
                const int cm = cel_at(su + K);
                const bool occupied = (unsigned)cm < (unsigned)f.ncell && ((wm >> cm) & 1ull);
                if (!occupied) {
                    const unsigned long long rest =
                        cells_up ? (cm >= 63 ? 0ull : wm >> (cm + 1))
                                 : (cm <= 0 ? 0ull : (cm >= 64 ? wm : wm & ((1ull << cm) - 1ull)));
                    if (rest == 0ull) break;
                    const int nx = cells_up ? cm + 1 + (int)__builtin_ctzll(rest) : 63 - (int)__builtin_clzll(rest);
                    su = entry_at(nx);
                    wdone = su >= wse;
                    continue;
                }
                int cl[K];
                int2 e[K];
                if constexpr (SC) {   // one base, constant offsets: the K entries merge into wide scalar loads
                    cint* tb = gtw + 2 * (su + K);
#pragma unroll
                    for (int k = 0; k < K; ++k) e[k] = make_int2(tb[2 * k], tb[2 * k + 1]);
                } else {
#pragma unroll
                    for (int k = 0; k < K; ++k) e[k] = tab_at(su + k + K);   // (su < wse <= S: entries to S + 2K - 1 exist)
                }
#pragma unroll
                for (int k = 0; k < K; ++k)   // (past the clip range: an offset no gather reaches, class 0)
                    if (su + k >= wse) e[k].x = INT32_MIN / 2;
#pragma unroll
                for (int k = 0; k < K; ++k)
                    cl[k] = (int)__builtin_amdgcn_ubfe(
                        (unsigned)__builtin_amdgcn_raw_buffer_load_b8(crs, fixedB + e[k].x, 0, 0), (unsigned)e[k].y,
                        (unsigned)f.cbits);
                if (STATS) {
                    ++st_iter;
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        const unsigned ld = act && e[k].x >= 0;
                        st_loads += ld; st_bytes += ld;
                    }
                }
                constexpr int G = kTfGroup < K ? kTfGroup : K;
#pragma unroll
                for (int k0 = 0; k0 < K; k0 += G) {
                    float4 cg[G];
#pragma unroll
                    for (int j = 0; j < G; ++j) cg[j] = s_tf[cl[k0 + j]];
#pragma unroll
                    for (int j = 0; j < G; ++j) {
                        r = fmaf(T, cg[j].x, r); g = fmaf(T, cg[j].y, g); bl = fmaf(T, cg[j].z, bl);
                        T = T * cg[j].w;
                    }
                }
                if (__all(!act || T < ert_eps_l)) break;
                su += K;
                wdone = su >= wse;
            }
        };
        if (lock_scalar) lock_march(std::true_type{});
        else lock_march(std::false_type{});
        if (!lane_ok) continue;
        r = r + T * f.bg[0]; g = g + T * f.bg[1]; bl = bl + T * f.bg[2];
        store_pixel(out, out_index(f.out_tiles, wt, x, y, f.H, f.tile_w, f.tile_h), f.out_rgb, r, g, bl);
        if (STATS == 2) count_work(stats, st_loads, st_bytes, st_iter * K);
        continue;
    }
    }   // LOCKV
    int s = F2B ? s_begin : s_end - 1;
    bool done = F2B ? (s >= s_end) : (s < s_begin);
    // general views, front to back: the empty-space test runs only after a batch that composited
    // nothing (T unchanged).  Inside tissue the test and its cell-distance load are skipped (wave-
    // uniformly when every lane is inside); skipping fewer alpha-0 samples is always exact.
    constexpr bool LAZY = ESS && !AXIS1 && (PREMUL || (!F2B && PTAB));
    bool ess_check = true;
    // the ERT threshold held in a VGPR across the loop: under the kernel's ~106 SGPRs the compiler
    // reloaded it from the kernel arguments every batch, an s_load + s_waitcnt lgkmcnt(0) that also
    // waited for the batch's outstanding TF reads (ISA, round 5)
    float ert_eps_v = f.ert_eps;
    asm volatile("" : "+v"(ert_eps_v));
    // RUNW on 64-bit volumes, front to back (C5): the next straight batch's two run words are loaded
    // while this batch composites (software pipelining; a jump or the ray's end leaves them unused,
    // the words are the same either way: bitwise the same frames)
#ifndef VR_RUNW_PREFETCH
#define VR_RUNW_PREFETCH 0
#endif
    constexpr bool PF = VR_RUNW_PREFETCH && RUNW && IDX64 && F2B && PREMUL;
    int64_t pf_qa = -1, pf_qb = -1;
    uint2 pf_wa = make_uint2(0u, 0u), pf_wb = make_uint2(0u, 0u);
    while (!done) {
        if (STATS) ++st_iter;
        const float T_batch = T;
        const float r_batch = r, g_batch = g, b_batch = bl;   // back to front: an alpha-0 batch leaves r, g, b
        if (ESS && AXIS1) {
            // whole empty run at once: the next occupied cell of the column in the direction of
            // travel (none: every later sample is alpha 0 -- the ray is finished).  Cells -1 / ncell
            // (outside the cube) are empty.
            const int cm = s_cel[s + K];
            const bool occupied = (unsigned)cm < (unsigned)f.ncell && ((colmask >> cm) & 1ull);
            if (F2B && PREMUL) {
                // without divergent control flow: every lane computes its jump target and takes it
                // when its cell is empty, then runs the batch.  A jump lands on the first sample of
                // the next occupied cell; a ray with none left moves to s = s_end, whose batch
                // composites only alpha-0 samples (an exact no-op) and then ends the ray.  Same
                // samples composited in the same order as the branchy form below.
                // (shift amounts clamped and results selected, so no lane-divergent branches; cm is
                // -1 .. ncell <= 64)
                unsigned long long rest;
                if (cells_up) {
                    const unsigned long long r = colmask >> min(cm + 1, 63);
                    rest = cm + 1 >= 64 ? 0ull : r;
                } else {
                    const unsigned long long r = colmask & ((1ull << min(max(cm, 0), 63)) - 1ull);
                    rest = cm <= 0 ? 0ull : (cm >= 64 ? colmask : r);
                }
                const int nx = cells_up ? cm + 1 + (int)__builtin_ctzll(rest) : 63 - (int)__builtin_clzll(rest);
                const int e = s_entry[rest == 0ull ? 0 : nx];
                // none left: s_end, past the ray's clip range, where every sample is TF(0) (alpha 0)
                const int sj = rest == 0ull ? s_end : e;
                if (STATS) st_jumps += !occupied;
                s = occupied ? s : sj;
            } else if (!occupied) {
                if (STATS) ++st_jumps;
                const unsigned long long rest =
                    cells_up ? (cm >= 63 ? 0ull : colmask >> (cm + 1))
                             : (cm <= 0 ? 0ull : (cm >= 64 ? colmask : colmask & ((1ull << cm) - 1ull)));
                if (rest == 0ull) { done = true; continue; }
                const int nxt = cells_up ? cm + 1 + __builtin_ctzll(rest) : 63 - __builtin_clzll(rest);
                s = s_entry[nxt];
                done = F2B ? (s >= s_end) : (s < s_begin);
                continue;
            }
        } else if (ESS && (!LAZY || ess_check)) {
            // jump over an empty macro cell before starting a batch
            int cell, cc[3] = {0, 0, 0};
            // a sample outside the unit cube has no cell of its own (its leaf index is clamped): no
            // jump from it.  Only the clip margin reaches there, when the dataset fills the cube
            // (L = 2^D, e.g. 512^3 / 2048^3).
            const bool in_cube = sample_cell(s, cell, cc);
            // Chebyshev distance dc > 0: the box of cells within dc - 1 of this one is empty; jump to
            // the first sample that may leave it (all earlier ones are alpha 0)
            // (a buffer load: 32-bit offset, no 64-bit address arithmetic; cell < ncell^3 always)
            const int dc = (f.edge_guard && !in_cube)
                               ? 0
                               : (int)__builtin_amdgcn_raw_buffer_load_b8(
                                     uniform_rsrc(cdist, f.ncell * f.ncell * f.ncell), cell, 0, 0);
            if (F2B && PREMUL) {
                // one jump per batch, taken by select (no divergent continue); the batch then starts
                // at the jump target, which may still lie in empty cells (alpha 0: exact no-ops)
                float sstar = 3.0e38f;
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    if (stp[c] == 0.0f) continue;
                    const bool up_axis = stp[c] > 0.0f;
                    const float bound = up_axis ? (float)(cc[c] + dc) * f.cell_q - f.shrink_q
                                                : (float)(cc[c] - dc + 1) * f.cell_q + f.shrink_q;
                    sstar = fminf(sstar, (bound - base[c]) * istp[c]);
                }
                const float nx = ceilf(sstar);
                const int sj = nx > (float)(s + 1) ? (nx < (float)f.S ? (int)nx : f.S) : s + 1;
                if (STATS) st_jumps += dc > 0;
                s = dc > 0 ? min(sj, s_end) : s;
            } else if (!F2B && !SHADE) {
                // the same, back to front: the jump lands on the last sample that may be inside
                // the empty box's far side in march order (or s_begin - 1: a batch of no-samples)
                float sstar = -3.0e38f;
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    if (stp[c] == 0.0f) continue;
                    const bool up_axis = stp[c] < 0.0f;
                    const float bound = up_axis ? (float)(cc[c] + dc) * f.cell_q - f.shrink_q
                                                : (float)(cc[c] - dc + 1) * f.cell_q + f.shrink_q;
                    sstar = fmaxf(sstar, (bound - base[c]) * istp[c]);
                }
                const float nx = floorf(sstar);
                const int sj = nx < (float)(s - 1) ? (nx > -1.0f ? (int)nx : -1) : s - 1;
                if (STATS) st_jumps += dc > 0;
                s = dc > 0 ? max(sj, s_begin - 1) : s;
            } else if (dc > 0) {
                if (STATS) ++st_jumps;
                float sstar = F2B ? 3.0e38f : -3.0e38f;
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    if (AXIS1 && c != ma) continue;
                    if (stp[c] == 0.0f) continue;
                    const bool up_axis = F2B ? (stp[c] > 0.0f) : (stp[c] < 0.0f);
                    const float bound = up_axis ? (float)(cc[c] + dc) * f.cell_q - f.shrink_q
                                                : (float)(cc[c] - dc + 1) * f.cell_q + f.shrink_q;
                    const float sc = (bound - base[c]) * istp[c];
                    sstar = F2B ? fminf(sstar, sc) : fmaxf(sstar, sc);
                }
                if (F2B) {
                    const float nx = ceilf(sstar);
                    s = nx > (float)(s + 1) ? (nx < (float)f.S ? (int)nx : f.S) : s + 1;
                    done = s >= s_end;
                } else {
                    const float nx = floorf(sstar);
                    s = nx < (float)(s - 1) ? (nx > -1.0f ? (int)nx : -1) : s - 1;
                    done = s < s_begin;
                }
                continue;
            }
        }
        // straight-line batch of K samples
        idx_t off[K];
        int cl[K];
        if (AXIS1 && !IDX64 && SPLIT) {
            // views along z with the split table: the ray's (x, y) offset is byte-aligned, so a
            // sample's class is the bfe at the entry's bit of byte fixedB + entry byte (the same byte
            // and bit as class_at of the summed bit offset; markers read class 0 out of range)
            if constexpr (SPLIT) {
                int2 e[K];
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    // one ds_read_b64 per entry: the compiler would pair adjacent entries into
                    // ds_read2_b64, 8 LDS cycles per pair instead of 2 + 2 (MI355X_MICROARCH LDS
                    // table) -- the table and TF reads keep the LDS pipe busy on this march
                    typedef const volatile __attribute__((address_space(3))) unsigned long long lds_u64;
                    const unsigned long long u = ((lds_u64*)(s_tab))[(F2B ? s + k : s - k) + K];
                    e[k] = make_int2((int)(uint32_t)u, (int)(uint32_t)(u >> 32));
                }
#pragma unroll
                for (int k = 0; k < K; ++k) off[k] = e[k].x;
                const int fixedB = (int)(fixed_off >> f.osh);
                const bool fast = ((ESS && PREMUL) || (PTAB && f.zero_transparent)) && f.cls0 == 0;
                if (fast) {
#pragma unroll
                    for (int k = 0; k < K; ++k)
                        cl[k] = (int)__builtin_amdgcn_ubfe(
                            (unsigned)__builtin_amdgcn_raw_buffer_load_b8(crs, fixedB + e[k].x, 0, 0), (unsigned)e[k].y,
                            (unsigned)f.cbits);
                } else {
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        const bool ok = (e[k].x | notin) >= 0;
                        const int v = (int)__builtin_amdgcn_ubfe(
                            (unsigned)__builtin_amdgcn_raw_buffer_load_b8(crs, ok ? fixedB + e[k].x : INT32_MIN, 0, 0),
                            (unsigned)e[k].y, (unsigned)f.cbits);
                        if (ESS) cl[k] = v + (ok ? 0 : (e[k].x == kTabNone ? n_tf : f.cls0));
                        else cl[k] = ok ? v : (e[k].x == kTabNone ? n_tf : f.cls0);
                    }
                }
                if (STATS) {
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        const unsigned ld = fast ? e[k].x >= 0 : (e[k].x | notin) >= 0;
                        st_loads += ld; st_bytes += ld;
                    }
                }
            }
        } else if (AXIS1 && !IDX64) {
            if constexpr (!SPLIT) {
            // table samples: kTabNone (outside [0, S)) reads the transparent slot n_tf; samples past
            // the ray's clip range are TF(0) there, alpha 0 whenever the clip is active.  Branch-free
            // gathers: an invalid sample's buffer offset is out of range, so the load returns 0
            // without a memory access, and the class is selected afterwards (no exec-mask branches).
#pragma unroll
            for (int k = 0; k < K; ++k) off[k] = s_tab[(F2B ? s + k : s - k) + K];
            const bool fast = ((ESS && PREMUL) || (PTAB && f.zero_transparent)) && f.cls0 == 0;
            // run words (RUNW): the batch's classes from two 8-byte loads.  A marker's word offset
            // ((fixed_off + marker) >> qsh) * 8 is negative -- out of range, a zero word -- and a marker
            // sample lies in word a / b only when that end is the same marker (a valid sample's word
            // index is >= 0), so it reads class 0 exactly as its own out-of-range load would.  A batch
            // with a sample in neither word on any lane loads per sample instead (exact either way).
            bool per_sample = true;
            if (RUNW) {
                int tk[K];
#pragma unroll
                for (int k = 0; k < K; ++k) tk[k] = (int)off[k] + zlow;
                const int qa = tk[0] >> f.qsh, qb = tk[K - 1] >> f.qsh;
                const auto wa = __builtin_amdgcn_raw_buffer_load_b64(crs, (int)((fixed_off + off[0]) >> f.qsh) * 8, 0, 0);
                const auto wb = __builtin_amdgcn_raw_buffer_load_b64(crs, (int)((fixed_off + off[K - 1]) >> f.qsh) * 8, 0, 0);
                bool miss = false;
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    miss |= run_miss(f, tk[k], qa, qb);
                    const int v = run_class(f, tk[k], qa, wa[0], wa[1], wb[0], wb[1]);
                    if (fast) {
                        cl[k] = v;
                    } else {
                        const bool ok = (off[k] | notin) >= 0;
                        cl[k] = ok ? v : (off[k] == kTabNone ? n_tf : f.cls0);
                    }
                }
                per_sample = __any(miss);
            }
            if (!per_sample) {
            } else if (fast) {
                // the common case, class 0 = TF(0) with alpha 0: a marker's offset fixed_off + marker is
                // already out of range, the load returns class 0, and TF(0) composites exactly like the
                // no-sample slot (both (0, 0, 0, 1) in the premultiplied table: front to back a no-op,
                // back to front r * 1 + 0 = r).  No selects at all: one add per sample.  Rays off the
                // dataset (!fixed_in) never get here (s_end = 0 whenever TF(0) is transparent).
#pragma unroll
                for (int k = 0; k < K; ++k) cl[k] = class_at(crs, f, (int)(fixed_off + off[k]));
            } else {
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const bool ok = (off[k] | notin) >= 0;
                    const int v = class_at(crs, f, ok ? (int)(fixed_off + off[k]) : INT32_MIN);
                    // ESS: v is 0 when !ok (out-of-range offset), so the sum selects without a branch
                    // (the load's result is used on both paths and cannot be sunk into an exec-masked
                    // block).  Exact mode keeps the sunk, exec-masked load: whole waves of invalid
                    // samples skip it there (measured: branch-free C3 ESS+ERT -4 %, C2 -14 %; exact +8 %).
                    if (ESS) cl[k] = v + (ok ? 0 : (off[k] == kTabNone ? n_tf : f.cls0));
                    else cl[k] = ok ? v : (off[k] == kTabNone ? n_tf : f.cls0);
                }
            }
            if (STATS) {   // run words: two 8-byte words per batch, plus the per-sample bytes of a fallback
                if (RUNW) { st_loads += 2; st_bytes += 16; }
                if (per_sample) {
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        const unsigned ld = fast ? off[k] >= 0 : (off[k] | notin) >= 0;
                        st_loads += ld; st_bytes += ld;
                    }
                }
            }
            }   // !SPLIT
        } else if (AXIS1) {
            if constexpr (!SPLIT) {
#pragma unroll
            for (int k = 0; k < K; ++k) off[k] = s_tab[(F2B ? s + k : s - k) + K];
            bool per_sample = true;
            if (RUNW) {
                // run words (above), as global loads: a batch end that is a marker (or a ray off the
                // dataset) loads word 0 instead, whose value no valid sample can select
                int tk[K];
#pragma unroll
                for (int k = 0; k < K; ++k) tk[k] = (int)off[k] + zlow;
                const int qa = tk[0] >> f.qsh, qb = tk[K - 1] >> f.qsh;
                const uint2* wp = reinterpret_cast<const uint2*>(cls);
                const int64_t ia = off[0] >= 0 && fixed_in ? (fixed_off + off[0]) >> f.qsh : 0;
                const int64_t ib = off[K - 1] >= 0 && fixed_in ? (fixed_off + off[K - 1]) >> f.qsh : 0;
                uint2 wa, wb;
                if (PF) {
                    wa = pf_wa;
                    wb = pf_wb;
                    if (ia != pf_qa) wa = wp[ia];
                    if (ib != pf_qb) wb = wp[ib];
                    const int sn = min(s + K, f.S);   // (table entries past S are kTabNone markers)
                    const int o0 = s_tab[sn + K], o1 = s_tab[sn + 2 * K - 1];
                    pf_qa = o0 >= 0 && fixed_in ? (fixed_off + o0) >> f.qsh : 0;
                    pf_qb = o1 >= 0 && fixed_in ? (fixed_off + o1) >> f.qsh : 0;
                    pf_wa = wp[pf_qa];
                    pf_wb = wp[pf_qb];
                } else {
                    wa = wp[ia];
                    wb = wp[ib];
                }
                bool miss = false;
                if (f.zspan2 && !__any((off[0] | off[K - 1]) < 0 || !fixed_in)) {
                    // host: a batch spans at most two z-bricks, i.e. two words; with both ends inside
                    // the dataset (the region is contiguous along z) every sample is valid and lies in
                    // the word of one of them -- no per-sample validity or miss tests
#pragma unroll
                    for (int k = 0; k < K; ++k) cl[k] = run_class(f, tk[k], qa, wa.x, wa.y, wb.x, wb.y);
                } else if (((ESS && PREMUL) || (PTAB && f.zero_transparent)) && f.cls0 == 0) {
                    // class 0 = TF(0) with alpha 0: a marker composites like the no-sample slot (the
                    // 32-bit fast path above), and rays off the dataset never march (s_end = 0)
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        const bool ok = off[k] >= 0;
                        miss |= ok && run_miss(f, tk[k], qa, qb);
                        const int v = run_class(f, tk[k], qa, wa.x, wa.y, wb.x, wb.y);
                        cl[k] = ok ? v : 0;
                    }
                } else {
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        const bool ok = off[k] >= 0 && fixed_in;
                        miss |= ok && run_miss(f, tk[k], qa, qb);
                        const int v = run_class(f, tk[k], qa, wa.x, wa.y, wb.x, wb.y);
                        cl[k] = ok ? v : (off[k] == kTabNone ? n_tf : f.cls0);
                    }
                }
                per_sample = __any(miss);
            }
            if (per_sample) {
#pragma unroll
                for (int k = 0; k < K; ++k)
                    cl[k] = (off[k] >= 0 && fixed_in) ? class_at64(cls, f, (int64_t)(fixed_off + off[k]))
                                                      : (off[k] == kTabNone ? n_tf : f.cls0);
            }
            if (STATS) {
                if (RUNW) { st_loads += 2; st_bytes += 16; }
                if (per_sample) {
#pragma unroll
                    for (int k = 0; k < K; ++k) { st_loads += off[k] >= 0; st_bytes += off[k] >= 0; }
                }
            }
            }   // !SPLIT
        } else if (!IDX64 && !SHADE && f.cls0 == 0 && f.mapout_ok &&
                   ((ESS && PREMUL) || (!CONIC && f.pad > 0))) {
            // General (orthographic or conic) ESS + ERT march -- and, with padded maps, every general
            // orthographic march (exact back to front, ESS alone, ERT alone) -- class 0 = TF(0),
            // class volume under 2^29 bytes: no per-sample exec-mask branch, so a batch's 3K
            // leaf-map reads issue together.  A sample outside the dataset sums at least one kMapOut
            // (a negative offset), one outside the cube is forced to kMapOut, and the buffer load
            // answers a negative offset with class 0 = TF(0) without touching memory.  TF(0) has
            // alpha 0 here (ESS requires it; the host sets a pad only with the clip, i.e. when TF(0)
            // is transparent), so it composites exactly like the no-sample slot: front to back
            // (0, 0, 0, 1) premultiplied, back to front r * (1 - 0) + c * 0 = r.  Same leaves and
            // classes as sample_off for every sample the exact march composites: the same frame bit
            // for bit.
            // q * 2^D computed directly in leaf units: multiplying by a power of two commutes with
            // round-to-nearest, so ((P0 + t dir) + 0.5) 2^D == (P0 2^D + t (dir 2^D)) + 2^(D-1) bit
            // for bit (an intermediate small enough to round differently as a denormal is absorbed
            // by the + 0.5; overflow and NaN land outside either way).  One multiply fewer per axis.
            const unsigned lim = (unsigned)(f.nleaf - 1);
            const float fs = (float)s;   // |s +- k| < 2^24: exact in float, = (float)(s +- k)
            const float hL = 0.5f * f.leaves;
            const uint32_t one_L = __float_as_uint(f.leaves);   // q < 1 <=> q 2^D < 2^D
            float P0L[3], dirL[3];
#pragma unroll
            for (int c = 0; c < 3; ++c) { P0L[c] = P0[c] * f.leaves; dirL[c] = dir[c] * f.leaves; }
            if (!CONIC && f.pad > 0 && (F2B ? s + K <= f.S : s >= K - 1)) {
                // padded leaf maps (orthographic, host-bounded): every sample of a batch that starts
                // in the clip range [s_begin, s_end] lies within f.pad leaves of the dataset box
                // (host: pad >= (K + 6) |step| 2^D + 4), so floor(q 2^D) indexes the padded maps
                // directly -- the padding's kMapOut IS the out-of-cube test (q < 0 included: floor,
                // not truncation), and no sample leaves [0, S).  Samples past the clip range are
                // outside the box along the axis that clipped them (kMapOut), TF(0) exactly as the
                // clipped march treats them.  Per sample: position, 3 floor-converts, 3 LDS reads,
                // one add3 -- no clamps or selects.
                // (v_cvt_flr_i32_f32 == (int)floorf on every float whose floor fits int32:
                // tools/microbench/cvt_flr_check.hip, exhaustive, 0 mismatches on MI355X.)  Oblique
                // C3 64 -> 52 us, orbit views 85 -> 70 us, frames bitwise unchanged (tools/ab_frames.py).
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const float t = (F2B ? fs + (float)k : fs - (float)k) * f.sd + f.fc;
                    const float qx = (P0L[0] + t * dirL[0]) + hL;
                    const float qy = (P0L[1] + t * dirL[1]) + hL;
                    const float qz = (P0L[2] + t * dirL[2]) + hL;
                    int ix, iy, iz;
                    asm("v_cvt_flr_i32_f32 %0, %1" : "=v"(ix) : "v"(qx));
                    asm("v_cvt_flr_i32_f32 %0, %1" : "=v"(iy) : "v"(qy));
                    asm("v_cvt_flr_i32_f32 %0, %1" : "=v"(iz) : "v"(qz));
                    off[k] = (int32_t)s_mx[ix] + s_my[iy] + s_mz[iz];
                }
            } else
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int sk = F2B ? s + k : s - k;
                const float t = (F2B ? fs + (float)k : fs - (float)k) * f.sd + f.fc;
                const float qx = (P0L[0] + t * dirL[0]) + hL;
                const float qy = (P0L[1] + t * dirL[1]) + hL;
                const float qz = (P0L[2] + t * dirL[2]) + hL;
                const unsigned ix = min((unsigned)(int)qx, lim);
                const unsigned iy = min((unsigned)(int)qy, lim);
                const unsigned iz = min((unsigned)(int)qz, lim);
                const int32_t o = (int32_t)s_mx[ix] + s_my[iy] + s_mz[iz];
                const bool in = max(max(__float_as_uint(qx), __float_as_uint(qy)), __float_as_uint(qz)) < one_L;
                off[k] = (in && (F2B ? sk < s_end : sk >= s_begin)) ? o : (int32_t)kMapOut;
            }
            const __amdgpu_buffer_rsrc_t grs = uniform_rsrc(cls, f.cls_bytes);
#pragma unroll
            for (int k = 0; k < K; ++k) {
                cl[k] = __builtin_amdgcn_raw_buffer_load_b8(grs, (int)off[k], 0, 0);   // (byte classes: host)
                if (STATS) { st_loads += off[k] >= 0; st_bytes += off[k] >= 0; }
            }
        } else if (!IDX64) {
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int sk = F2B ? s + k : s - k;
                int cell, cc[3];
                off[k] = sample_off(sk, cell, cc);
                const bool valid = F2B ? (sk < s_end) : (sk >= s_begin);
                if (!valid) off[k] = -2;
            }
            const __amdgpu_buffer_rsrc_t grs = uniform_rsrc(cls, f.cls_bytes);
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const bool ok = off[k] >= 0;
                const int v = __builtin_amdgcn_raw_buffer_load_b8(grs, ok ? (int)off[k] : INT32_MIN, 0, 0);
                cl[k] = ok ? v : (off[k] == -2 ? n_tf : f.cls0);   // general views: the sunk form measured best
                if (STATS) { st_loads += ok; st_bytes += ok; }
            }
        } else {
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int sk = F2B ? s + k : s - k;
                int cell, cc[3];
                off[k] = sample_off(sk, cell, cc);
                const bool valid = F2B ? (sk < s_end) : (sk >= s_begin);
                if (!valid) off[k] = -2;
            }
#pragma unroll
            for (int k = 0; k < K; ++k) {
                cl[k] = off[k] >= 0 ? class_at64(cls, f, (int64_t)off[k]) : (off[k] == -2 ? n_tf : f.cls0);
                if (STATS) { st_loads += off[k] >= 0; st_bytes += off[k] >= 0; }
            }
        }
        // Branch-free composite: a sample outside the range (class n_tf) or with alpha 0 contributes
        // w = 0 and (1 - 0) = 1, which leaves r, g, b, T bit-for-bit unchanged (colours are finite).
        if (PREMUL) {
            // TF reads issued in groups of G before the group's composite (LDS latency once per group)
            constexpr int G = kTfGroup < K ? kTfGroup : K;
#pragma unroll
            for (int k0 = 0; k0 < K; k0 += G) {
                if (!AXIS1 && f.c0_noop) {
                    // general views: a group in which every lane's samples are class 0 -- alpha 0, the
                    // premultiplied entry (0, 0, 0, 1): r + T 0 = r, T 1 = T -- composites nothing:
                    // the wave skips its TF reads (LDS cycles) and fmas.  (Oblique C3 -5 %; axis views
                    // +7-14 %: their batches are rarely blank wave-wide, so it is off there.)
                    int any = 0;
#pragma unroll
                    for (int j = 0; j < G; ++j) any |= cl[k0 + j];
                    if (!__any(any != 0)) continue;
                }
                float4 cg[G];
#pragma unroll
                for (int j = 0; j < G; ++j) cg[j] = s_tf[cl[k0 + j]];
#pragma unroll
                for (int j = 0; j < G; ++j) {
                    r = fmaf(T, cg[j].x, r); g = fmaf(T, cg[j].y, g); bl = fmaf(T, cg[j].z, bl);
                    T = T * cg[j].w;
                }
            }
        } else if (!F2B && PTAB) {
            constexpr int G = kTfGroup < K ? kTfGroup : K;
#pragma unroll
            for (int k0 = 0; k0 < K; k0 += G) {
                float4 cg[G];
#pragma unroll
                for (int j = 0; j < G; ++j) cg[j] = s_tf[cl[k0 + j]];
#pragma unroll
                for (int j = 0; j < G; ++j) {   // r * (1 - a) + c * a, both products from the table
                    r = r * cg[j].w + cg[j].x; g = g * cg[j].w + cg[j].y; bl = bl * cg[j].w + cg[j].z;
                }
            }
        } else {   // shaded samples (SHADE: the colour is shaded per sample, the table is plain rgba)
#pragma unroll
        for (int k = 0; k < K; ++k) {
            float4 col = s_tf[cl[k]];
            const float a = col.w;
            if (SHADE && off[k] >= 0 && (!AXIS1 || fixed_in) && a != 0.0f) {
                // the shaded sample's normal, addressed through the raw leaf -> voxel maps
                const int sk = F2B ? s + k : s - k;
                const float t = (float)sk * f.sd + f.fc;
                const float qx = (P0[0] + t * dir[0]) + 0.5f;
                const float qy = (P0[1] + t * dir[1]) + 0.5f;
                const float qz = (P0[2] + t * dir[2]) + 0.5f;
                const int ix = (int)(qx * f.leaves), iy = (int)(qy * f.leaves), iz = (int)(qz * f.leaves);
                const int64_t c = (int64_t)s_raw[ix] * f.d2i * f.d3i + (int64_t)s_raw[f.nleaf + iy] * f.d3i +
                                  s_raw[2 * f.nleaf + iz];
                shade_normal(reinterpret_cast<const float4*>(vol)[c], Lh, f.ka, f.kd, f.ks, f.shininess, col.x,
                             col.y, col.z);
            }
            if (F2B) {
                const float w = T * a;
                // fused: front-to-back is already a reassociation within the ERT tolerance
                r = fmaf(w, col.x, r); g = fmaf(w, col.y, g); bl = fmaf(w, col.z, bl);
                T = T * (1.0f - a);
            } else {
                r = r * (1 - a) + col.x * a;
                g = g * (1 - a) + col.y * a;
                bl = bl * (1 - a) + col.z * a;
            }
        }
        }
        if (LAZY) ess_check = F2B ? T == T_batch : (r == r_batch && g == g_batch && bl == b_batch);
        // early ray termination, checked once per batch: what a batch adds after T < eps is <= eps
        if (F2B && T < ert_eps_v) done = true;
        s = F2B ? s + K : s - K;
        if (F2B ? (s >= s_end) : (s < s_begin)) done = true;
    }
    if (F2B) { r = r + T * f.bg[0]; g = g + T * f.bg[1]; bl = bl + T * f.bg[2]; }
    store_pixel(out, out_index(f.out_tiles, wt, x, y, f.H, f.tile_w, f.tile_h), f.out_rgb, r, g, bl);
    // counting pass (vr_count_work): class gathers that touched memory, their bytes and the samples
    // evaluated (batches x K) of this ray, summed over the frame
    if (STATS == 2) count_work(stats, st_loads, st_bytes, st_iter * K);
    if (STATS == 1) {   // diagnostic build only (VR_STATS=1): plain stores, no atomics (low distortion)
        // per wave (6 words, every lane stores the same wave-uniform values): t_entry, after the
        // staging barrier, after the table barrier, t_start (prologue done), t_end, xcc; per lane
        // (2 words, after the nw * 6 wave words): iters | loads << 32, jumps | 1 << 63
        const unsigned wave_id = blk * 4 + (threadIdx.x >> 6);
        const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();
        unsigned xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        unsigned long long* ws = stats + 6 * (size_t)wave_id;
        ws[0] = t_entry; ws[1] = t_b1; ws[2] = t_b2; ws[3] = t_start; ws[4] = t_end; ws[5] = xcc & 0xf;
        unsigned long long* ls = stats + 6 * (size_t)gridDim.x * 4 + 2 * ((size_t)wave_id * 64 + (threadIdx.x & 63));
        ls[0] = (unsigned long long)st_iter | ((unsigned long long)st_loads << 32);
        ls[1] = (unsigned long long)st_jumps | (1ull << 63);
    }
    }   // slot loop
}

// must match the kernel's LDS carve-up (vrc_march_kernel prologue)
static size_t vrc_lds_bytes(const VrcFrame& f, int n_tf, bool idx64, int K) {
    const bool shade = (f.flags & 8) != 0;
    const bool axis1 = f.axis1 >= 0 && !f.conic;
    size_t b = (size_t)(n_tf + 1) * sizeof(float4);
    const size_t span = (size_t)f.nleaf + 2 * (size_t)f.pad;   // general views: padded leaf maps
    b += axis1 ? (size_t)f.nleaf * 4 : span * (idx64 ? 8 : 4) + 2 * span * 4;
    if (shade) b += (size_t)3 * f.nleaf * 4;
    if (axis1) {
        const size_t n_tab = (size_t)f.S + 2 * K;
        b += (n_tab * (f.tsplit ? 8 : 4) + (size_t)f.ncell * 4 + n_tab + 3) & ~(size_t)3;   // whole words (staged as int32)
        b += 16;   // the table is staged in whole int4s: up to 12 B past its end
    }
    return b;
}

// samples per straight-line batch: batch 0 = the measured default, K = 8 whenever empty-space
// skipping is on (every view: C3 ESS + ERT 29.1 -> 28.5 us, S = 250 28.9 -> 27.2 us, C3 exact with
// empty cells skipped 58.8 -> 55.3 us, C2 exact 21.6 -> 21.0 us, oblique exact 79 -> 78 us; C2 ESS +
// ERT 14.6 -> 14.9 us is the one loss) and for conic views; K = 16 for the marches that skip
// nothing (ERT alone, an opaque TF(0)); SHADE always 8.  (Axis-aligned front-to-back marches of
// 1000 samples or more took K = 16 until the leaf-column masks: with them C4 S = 1024 K = 8 20.9
// vs K = 16 24.7 us, C5 46,800 vs 42,600 Mrays/s; round 5.)
static int vrc_batch(const VrcFrame& f, int batch) {
    if (f.flags & 8) return 8;
    if (batch == 0) {
        const bool ess = (f.flags & 1) && f.zero_transparent;
        return (ess || f.conic) ? 8 : 16;
    }
    return batch >= 16 ? 16 : 8;
}

// bytes of the published AXIS1 view table (march LDS layout: tab | entry | cel), 0 if the frame has none
int vrc_batch_of(const VrcFrame& f, int batch) { return vrc_batch(f, batch); }

size_t vrc_axis1_table_bytes(const VrcFrame& f, int batch) {
    if (f.axis1 < 0 || f.conic) return 0;
    const int K = vrc_batch(f, batch);
    const size_t n_tab = (size_t)f.S + 2 * K;
    return (n_tab * (f.tsplit ? 8 : 4) + (size_t)f.ncell * 4 + n_tab + 3) & ~(size_t)3;
}

template <int STATS, int K>
static void launch_vrc_variant(const VrcFrame& f, const WorkTile* work, const int32_t* order, int n_blocks_in,
                               const uint8_t* cls, const int32_t* maps, const int64_t* mapx64, const uint32_t* occ,
                               const float4* tf, int n_tf, float4* out, unsigned long long* stats, hipStream_t st,
                               const float* vol, const int32_t* rawmaps, const unsigned long long* occcol,
                               const uint8_t* cdist, const int32_t* gtab, int32_t* gtab_out) {
    const bool f2b = (f.flags & 2) != 0, ess = (f.flags & 1) != 0 && f.zero_transparent;
    const bool shade = (f.flags & 8) != 0;
    const bool idx64 = mapx64 != nullptr, ax1 = f.axis1 >= 0;
    const size_t lds = vrc_lds_bytes(f, n_tf, idx64, K);
    // f.persist_wgs > 0: persistent grid of 256 CUs x persist_wgs workgroups (multiple of 8)
    int n_blocks = n_blocks_in;
    if (f.persist_wgs > 0) n_blocks = std::min(n_blocks_in, 256 * f.persist_wgs);
#define VR_L(F2B_, ESS_, I64_, AX_, SH_)                                                                    \
    hipLaunchKernelGGL((vrc_march_kernel<F2B_, ESS_, I64_, AX_, K, SH_, STATS>), dim3(n_blocks), dim3(kWgThreads), \
                       lds, st, f, work, order, cls, maps, mapx64, occ, tf, n_tf, out, stats, vol, rawmaps, occcol, cdist, gtab, gtab_out)
#define VR_L2(I64_, AX_, SH_)                                                                            \
    if (f2b) { if (ess) VR_L(true, true, I64_, AX_, SH_); else VR_L(true, false, I64_, AX_, SH_); } \
    else { if (ess) VR_L(false, true, I64_, AX_, SH_); else VR_L(false, false, I64_, AX_, SH_); }
    const int geom = f.conic ? kGeomConic
                             : (ax1 ? (f.zrun && !shade ? kGeomAxis1Run
                                                        : (f.tsplit && !shade && !idx64 ? kGeomAxis1Z : kGeomAxis1))
                                    : kGeomOrtho);
    if (shade) {
        if (geom == kGeomConic) { if (idx64) { VR_L2(true, kGeomConic, true) } else { VR_L2(false, kGeomConic, true) } }
        else if (geom == kGeomAxis1) { if (idx64) { VR_L2(true, kGeomAxis1, true) } else { VR_L2(false, kGeomAxis1, true) } }
        else if (idx64) { VR_L2(true, kGeomOrtho, true) } else { VR_L2(false, kGeomOrtho, true) }
    } else if (idx64) {
        if (geom == kGeomAxis1) { VR_L2(true, kGeomAxis1, false) }
        else if (geom == kGeomAxis1Run) { VR_L2(true, kGeomAxis1Run, false) }
        else if (geom == kGeomConic) { VR_L2(true, kGeomConic, false) }
        else { VR_L2(true, kGeomOrtho, false) }
    } else {
        if (geom == kGeomAxis1) { VR_L2(false, kGeomAxis1, false) }
        else if (geom == kGeomAxis1Run) { VR_L2(false, kGeomAxis1Run, false) }
        else if (geom == kGeomAxis1Z) { VR_L2(false, kGeomAxis1Z, false) }
        else if (geom == kGeomConic) { VR_L2(false, kGeomConic, false) }
        else { VR_L2(false, kGeomOrtho, false) }
    }
#undef VR_L2
#undef VR_L
}

hipError_t launch_vrc_stats(const VrcFrame& f, const WorkTile* work, const int32_t* order, int n_blocks,
                            const uint8_t* cls, const int32_t* maps, const uint32_t* occ, const float4* tf,
                            int n_tf, float4* out, unsigned long long* stats, hipStream_t st,
                            const unsigned long long* occcol, const uint8_t* cdist, const int32_t* gtab) {
    launch_vrc_variant<1, 16>(f, work, order, n_blocks, cls, maps, nullptr, occ, tf, n_tf, out, stats, st, nullptr,
                                 nullptr, occcol, cdist, gtab, nullptr);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// Exact count of samples whose leaf lies inside the dataset (Octree.cu:91-94), N_in of SURVEY 8(d).
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void vrc_count_kernel(VrcFrame f, const WorkTile* __restrict__ work,
                                                        const int32_t* __restrict__ gmaps,
                                                        unsigned long long* __restrict__ total) {
    const WorkTile wt = work[blockIdx.x];
    int x, y;
    ray_of_thread(wt, x, y);
    unsigned long long n = 0;
    if (x < f.W && y < f.H) {
        float P0[3], dir[3], fb[3], stp[3], istp[3];
        int u0, u1;
        if (f.conic) ray_setup<true>(f, x, y, P0, dir, fb, stp, istp, u0, u1);
        else ray_setup<false>(f, x, y, P0, dir, fb, stp, istp, u0, u1);
        double bd[3], sdd[3];
        for (int c = 0; c < 3; ++c) {
            bd[c] = ((double)P0[c] + (double)f.fc * dir[c]) + 0.5;
            sdd[c] = (double)f.sd * dir[c];
        }
        int s0, s1;
        clip_range(bd, sdd, f.box_lo, f.box_hi, f.S, s0, s1);
        for (int s = s0; s < s1; ++s) {
            const float t = (float)s * f.sd + f.fc;
            const float qx = (P0[0] + t * dir[0]) + 0.5f;
            const float qy = (P0[1] + t * dir[1]) + 0.5f;
            const float qz = (P0[2] + t * dir[2]) + 0.5f;
            if (!(qx >= 0.0f && qx < 1.0f && qy >= 0.0f && qy < 1.0f && qz >= 0.0f && qz < 1.0f)) continue;
            const int ix = (int)(qx * f.leaves), iy = (int)(qy * f.leaves), iz = (int)(qz * f.leaves);
            if ((gmaps[ix] | gmaps[f.nleaf + iy] | gmaps[2 * f.nleaf + iz]) >= 0) ++n;
        }
    }
    // wave reduction, one atomic per wave
    for (int o = 32; o > 0; o >>= 1) n += __shfl_down(n, o, 64);
    if ((threadIdx.x & 63) == 0 && n) atomicAdd(total, n);
}

// ------------------------------------------------------------------------------------------------
// Tile assembly on the gathering rank: compact per-rank tile blocks -> x-major frame.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ float4 load_tile_pixel(const float4* tiles, int64_t idx, bool rgb) {
    if (!rgb) return tiles[idx];
    const float* t = reinterpret_cast<const float*>(tiles) + idx * 3;
    return make_float4(t[0], t[1], t[2], 1.0f);
}

template <bool RGB>
__global__ __launch_bounds__(256) void assemble_kernel(int W, int H, int tile_w, int tile_h, int ntx,
                                                       int nty, int n_ranks, int max_tiles,
                                                       const float4* __restrict__ tiles,
                                                       float4* __restrict__ frame) {
    const int64_t px = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t per_tile = (int64_t)tile_w * tile_h;
    const int64_t total = (int64_t)n_ranks * max_tiles * per_tile;
    if (px >= total) return;
    const int64_t slot_g = px / per_tile;
    const int within = (int)(px % per_tile);
    const int rank = (int)(slot_g / max_tiles), k = (int)(slot_g % max_tiles);
    const int64_t t = (int64_t)rank + (int64_t)k * n_ranks;
    if (t >= (int64_t)ntx * nty) return;
    const int tx = (int)(t / nty), ty = (int)(t % nty);
    const int i = within / tile_h, j = within % tile_h;
    const int x = tx * tile_w + i, y = ty * tile_h + j;
    if (x >= W || y >= H) return;
    frame[(int64_t)x * H + y] = load_tile_pixel(tiles, px, RGB);
}

// Frame assembly over a tile list: every frame pixel, in frame order (coalesced stores), copies
// its tile's gathered pixel when the tile was rendered (slot_of[t] >= 0: block index in the
// gathered buffer) and otherwise writes the background, which is what the march yields there.
template <bool RGB>
// blockIdx.y = frame of a batch: its own slot map (map_stride entries further) and frame (W*H further).
__global__ __launch_bounds__(256) void assemble_list_kernel(int W, int H, int tile_w, int tile_h, int nty,
                                                            const int32_t* __restrict__ slot_of,
                                                            const float4* __restrict__ tiles, float4 bg,
                                                            float4* __restrict__ frame, int64_t map_stride) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)W * H) return;
    slot_of += blockIdx.y * map_stride;
    frame += blockIdx.y * (int64_t)W * H;
    const int x = (int)(i / H), y = (int)(i % H);
    const int slot = slot_of[(x / tile_w) * nty + y / tile_h];
    store_f4(frame + i, slot < 0 ? bg : load_tile_pixel(tiles, (int64_t)slot * tile_w * tile_h + (x % tile_w) * tile_h + (y % tile_h), RGB));
}

// ------------------------------------------------------------------------------------------------
// Whole-frame work list on the device (moving cameras: the culled rectangle changes every frame, so
// a host-built list would cost a host build + a synchronous upload per frame).  Same list as the
// host's work_for for the diagonal XCD deal: position 8 j + x holds XCD group x's j-th visible work
// tile (group (tx + ty) % 8, each group walking its tiles column by column), holes are tiles far off
// screen, then every work tile outside the visible rectangle in x-major order with slot = -1 (the
// march stores the background there).  One workgroup.
// ------------------------------------------------------------------------------------------------
__host__ __device__ inline int rows_with_residue(int a, int b, int r) {   // #ty in [a, b] with ty % 8 == r
    if (b < a) return 0;
    const int first = a + ((r - a) % 8 + 8) % 8;
    return first > b ? 0 : (b - first) / 8 + 1;
}

// columns of group x (tx % 8 == x) in [tx0, tx0 + dc): the column deal's whole-column groups
__host__ __device__ inline int cols_of_group(int x, int tx0, int dc) {
    return dc <= 0 ? 0 : rows_with_residue(tx0, tx0 + dc - 1, x);
}

// tiles of group x in the columns [tx0, tx0 + dc) of a rectangle with rows [ty0, ty1]; deal 1 (column
// interleave): group x holds whole columns tx % 8 == x
__host__ __device__ inline int group_count(int x, int tx0, int dc, int ty0, int ty1, int deal = 0) {
    if (deal == 1) return cols_of_group(x, tx0, dc) * (ty1 - ty0 + 1);
    int n = (ty1 - ty0 + 1) * (dc / 8);   // 8 consecutive columns give every group one tile per row
    for (int r = 0; r < dc % 8; ++r) {
        const int col = tx0 + 8 * (dc / 8) + r;
        n += rows_with_residue(ty0, ty1, ((x - col) % 8 + 8) % 8);
    }
    return n;
}

// One thread per frame tile (and per dealt slot): the visible tile (tx, ty) goes to slot 8j + x of
// XCD group x = (tx + ty) mod 8, j = its index in that group's column-major walk (closed form); a
// slot past its group's count is a hole (a no-op entry); a culled tile goes after the slots, in
// frame order.  Every entry is written exactly once, so no barrier: many workgroups, one round of
// stores (the single-workgroup form took ~25 us per rebuild under a concurrent march).
// The cell columns (along the view axis) the rays of work tile (tx, ty) can reach: the rays' q range
// over the tile's corner pixels (q is affine in the pixel), one leaf of margin -- the same test as
// the host's visible_tiles for farm tiles.  True when none of them holds an occupied cell.
__device__ bool tile_columns_empty(const WlCull& c, int tx, int ty) {
    const int px0 = tx * kWgRaysX, px1 = min(c.W, (tx + 1) * kWgRaysX) - 1;
    const int py0 = ty * kWgRaysY, py1 = min(c.H, (ty + 1) * kWgRaysY) - 1;
    const double L = (double)c.nleaf;
    int lo[2], hi[2];
    for (int k = 0; k < 2; ++k) {
        double qmin = 1e300, qmax = -1e300;
        for (int cx = 0; cx < 2; ++cx)
            for (int cy = 0; cy < 2; ++cy) {
                const double x = cx ? px1 : px0, y = cy ? py1 : py0;
                const double q = c.tl[k] + (x * c.rsw / c.W) * c.right[k] + (y * c.rsh / c.H) * -c.up[k] + 0.5;
                qmin = fmin(qmin, q); qmax = fmax(qmax, q);
            }
        const double l0 = floor(qmin * L) - 1.0, l1 = floor(qmax * L) + 1.0;
        if (!(l1 >= 0.0 && l0 <= L - 1.0)) return true;   // outside the cube on this axis: TF(0) only
        lo[k] = (int)fmax(0.0, l0) >> c.cb_shift;
        hi[k] = (int)fmin(L - 1.0, l1) >> c.cb_shift;
    }
    const int32_t* S = c.sat;
    const int n = S[(hi[0] + 1) * c.side + hi[1] + 1] - S[lo[0] * c.side + hi[1] + 1] - S[(hi[0] + 1) * c.side + lo[1]] +
                  S[lo[0] * c.side + lo[1]];
    return n == 0;
}

__global__ __launch_bounds__(256) void worklist_kernel(int ntx, int nty, int tx0, int tx1, int ty0, int ty1,
                                                       int n_slots, WorkTile* __restrict__ out, WlCull cull,
                                                       int deal) {
    const int w = tx1 >= tx0 ? tx1 - tx0 + 1 : 0, h = ty1 >= ty0 ? ty1 - ty0 + 1 : 0;
    const int t = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (t < n_slots) {
        const int x = t & 7, j = t >> 3;
        const int cnt = w > 0 ? group_count(x, tx0, w, ty0, ty1, deal) : 0;
        if (j >= cnt) out[t] = WorkTile{1 << 30, 1 << 30, 0, 0};
    }
    if (t < ntx * nty) {
        const int tx = t / nty, ty = t % nty;
        const bool in_col = tx >= tx0 && tx <= tx1;
        if (in_col && ty >= ty0 && ty <= ty1) {
            // deal 0: group (tx + ty) % 8, walked column by column; deal 1: group tx % 8 (whole
            // columns), j = the tile's index in its group's column-major walk either way
            const int x = deal == 1 ? (tx & 7) : ((tx + ty) & 7);
            const int j = deal == 1 ? cols_of_group(x, tx0, tx - tx0) * h + (ty - ty0)
                                    : group_count(x, tx0, tx - tx0, ty0, ty1) +
                                          rows_with_residue(ty0, ty - 1, ((x - tx) % 8 + 8) % 8);
            // a tile whose rays meet only empty columns keeps its slot but is marked culled: the march
            // stores its background without staging anything
            const int slot = (cull.sat && tile_columns_empty(cull, tx, ty)) ? -1 : 0;
            out[8 * j + x] = WorkTile{tx * kWgRaysX, ty * kWgRaysY, slot, 0};
        } else {
            const int before = min(max(tx - tx0, 0), w) * h + (in_col ? min(max(ty - ty0, 0), h) : 0);
            out[n_slots + t - before] = WorkTile{tx * kWgRaysX, ty * kWgRaysY, -1, 0};
        }
    }
}

hipError_t launch_worklist(int ntx, int nty, int tx0, int tx1, int ty0, int ty1, int n_slots, WorkTile* out,
                           const WlCull& cull, int deal, hipStream_t st) {
    const int n = max(n_slots, ntx * nty);
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(worklist_kernel, dim3((n + 255) / 256), dim3(256), 0, st, ntx, nty, tx0, tx1, ty0, ty1, n_slots,
                       out, cull, deal);
    return hipGetLastError();
}

// visible rectangle -> (slots of the dealt part, total work tiles) for worklist_kernel
void worklist_size(int ntx, int nty, int tx0, int tx1, int ty0, int ty1, int* n_slots, int* n_total, int deal) {
    const int w = tx1 >= tx0 ? tx1 - tx0 + 1 : 0;
    int slots = 0;
    for (int x = 0; x < 8; ++x) {
        const int cnt = w > 0 ? group_count(x, tx0, w, ty0, ty1, deal) : 0;
        if (cnt > 0) slots = max(slots, 8 * (cnt - 1) + x + 1);
    }
    const int h = ty1 >= ty0 ? ty1 - ty0 + 1 : 0;
    *n_slots = slots;
    *n_total = slots + ntx * nty - w * h;
}

// Multi-GPU rank 0: the peers' gathered RGB tiles into the frames rank 0 has already marched its own
// tiles (and the background) into.  One lane per tile pixel, consecutive lanes along y: consecutive
// frame addresses.  map[2b], map[2b + 1] = user tile (x-major, tile x tile) and frame of block b.
__global__ __launch_bounds__(256) void scatter_tiles_kernel(int W, int H, int tile, int nty,
                                                            const int32_t* __restrict__ map, int64_t n,
                                                            const float* __restrict__ tiles,
                                                            float4* __restrict__ frames) {
    const int64_t px = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t per = (int64_t)tile * tile;
    if (px >= n * per) return;
    const int64_t b = px / per;
    const int32_t t = map[2 * b], f = map[2 * b + 1];
    const int within = (int)(px % per);
    const int x = (t / nty) * tile + within / tile, y = (t % nty) * tile + within % tile;
    if (x >= W || y >= H) return;
    const float* s = tiles + px * 3;
    store_f4(frames + (int64_t)f * W * H + (int64_t)x * H + y, make_float4(s[0], s[1], s[2], 1.0f));
}

// Multi-GPU plan on the device (vr_multi.cpp group_render).  The host decides the frame's tile
// owners (visible tiles dealt to the ranks, -1 = a tile that can hold only background) and the
// per-rank counts it needs for the RCCL transfer sizes; this kernel expands them into this part's
// work list -- rank 0: its own tiles' 16 x 16 work tiles (slot 0, marched into the frame), then the
// invisible tiles' work tiles (slot -1, background); a peer: its own tiles' work tiles with the
// compact-buffer slot k = the tile's index among this rank's tiles -- and, on rank 0, the scatter
// map of the peers' tiles (block mbase[f, q] + k holds tile t of frame f).  Every tile's entries are
// placed by exclusive prefix sums over the tiles in ascending id, the order the host deal and the
// peers' buffers use, so the frame is the one the host-built lists gave (bitwise: a work list's
// order changes no pixel).  One workgroup per frame of the batch; no host upload but the owners.
__device__ __forceinline__ int block_excl_scan(int v, int* s_w, int& total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) s_w[w] = x;
    __syncthreads();
    int off = 0;
    total = 0;
#pragma unroll
    for (int i = 0; i < kWgThreads / 64; ++i) {
        off += i < w ? s_w[i] : 0;
        total += s_w[i];
    }
    __syncthreads();
    return off + x - v;
}

__global__ __launch_bounds__(256) void plan_kernel(const int8_t* __restrict__ owner, int ntiles, int nty, int W, int H,
                                                   int T, int rank, int n_ranks, const int32_t* __restrict__ woff,
                                                   const int32_t* __restrict__ nown, const int32_t* __restrict__ mbase,
                                                   WorkTile* __restrict__ work, int32_t* __restrict__ map) {
    __shared__ int s_w[kWgThreads / 64];
    const int f = blockIdx.x;
    const int8_t* own = owner + (size_t)f * ntiles;
    WorkTile* wl = work + woff[f];
    const int bg_base = rank == 0 ? nown[f] : 0;   // rank 0: first background entry of the frame
    int c_mine = 0, c_wt = 0, c_bg = 0;            // running totals of the chunks before
    const int per = T / kWgRaysX;                  // work tiles per tile edge (T is a multiple of 16)
    for (int t0 = 0; t0 < ntiles; t0 += kWgThreads) {
        const int t = t0 + (int)threadIdx.x;
        const int o = t < ntiles ? (int)own[t] : -2;
        const int tx = t / nty, ty = t % nty;
        // the tile's work tiles inside the frame
        const int nx = t < ntiles ? min(per, (W - tx * T + kWgRaysX - 1) / kWgRaysX) : 0;
        const int ny = t < ntiles ? min(per, (H - ty * T + kWgRaysY - 1) / kWgRaysY) : 0;
        const int wt = nx * ny;
        const bool mine = o == rank, bg = rank == 0 && o == -1;
        int tot;
        const int k = block_excl_scan(mine ? 1 : 0, s_w, tot) + c_mine;
        c_mine += tot;
        const int e_mine = block_excl_scan(mine ? wt : 0, s_w, tot) + c_wt;
        c_wt += tot;
        const int e_bg = block_excl_scan(bg ? wt : 0, s_w, tot) + c_bg;
        c_bg += tot;
        if (mine || bg) {
            const int base = mine ? e_mine : bg_base + e_bg;
            const int slot = rank == 0 ? (mine ? 0 : -1) : k;
            for (int i = 0; i < nx; ++i)
                for (int j = 0; j < ny; ++j) {
                    const int ox = i * kWgRaysX, oy = j * kWgRaysY;
                    wl[base + i * ny + j] = WorkTile{tx * T + ox, ty * T + oy, slot, rank == 0 ? 0 : ((ox << 16) | oy)};
                }
        }
    }
    if (rank == 0)   // the peers' tiles: (tile, frame) at their receive blocks, peer by peer
        for (int q = 1; q < n_ranks; ++q) {
            int c = 0;
            for (int t0 = 0; t0 < ntiles; t0 += kWgThreads) {
                const int t = t0 + (int)threadIdx.x;
                const bool his = t < ntiles && (int)own[t] == q;
                int tot;
                const int kq = block_excl_scan(his ? 1 : 0, s_w, tot) + c;
                c += tot;
                if (his) {
                    const int b = mbase[(size_t)f * n_ranks + q] + kq;
                    map[2 * b] = t;
                    map[2 * b + 1] = f;
                }
            }
        }
}

hipError_t launch_plan(const int8_t* owner, int n_frames, int ntiles, int nty, int W, int H, int tile, int rank,
                       int n_ranks, const int32_t* woff, const int32_t* nown, const int32_t* mbase, WorkTile* work,
                       int32_t* map, hipStream_t st) {
    if (n_frames <= 0 || ntiles <= 0) return hipSuccess;
    hipLaunchKernelGGL(plan_kernel, dim3(n_frames), dim3(kWgThreads), 0, st, owner, ntiles, nty, W, H, tile, rank,
                       n_ranks, woff, nown, mbase, work, map);
    return hipGetLastError();
}

hipError_t launch_scatter_tiles(int W, int H, int tile, const int32_t* map, int n_tiles, const float* tiles,
                                float4* frames, hipStream_t st) {
    const int64_t total = (int64_t)n_tiles * tile * tile;
    if (total == 0) return hipSuccess;
    const int nty = (H + tile - 1) / tile;
    hipLaunchKernelGGL(scatter_tiles_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, W, H, tile, nty,
                       map, (int64_t)n_tiles, tiles, frames);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// Launch wrappers (called from vr_api.cpp)
// ------------------------------------------------------------------------------------------------
hipError_t launch_classify(const float* vol, int64_t n, float max_intensity, double cal_max,
                           const float* lo, const float* hi, int n_tf, uint8_t* cls_vrc,
                           uint8_t* cls_test, const int64_t* lay, int64_t d2, int64_t d3, hipStream_t st) {
    const int64_t blocks64 = (n + 255) / 256;
    const int blocks = (int)(blocks64 < 65536 ? blocks64 : 65536);
    hipLaunchKernelGGL(classify_kernel, dim3(blocks), dim3(256), 0, st, vol, n, max_intensity, cal_max,
                       lo, hi, n_tf, cls_vrc, cls_test, lay, d2, d3);
    return hipGetLastError();
}

hipError_t launch_cell_dist(const unsigned long long* occ, int ncell, int cap, uint8_t* a, uint8_t* b, uint8_t** result,
                            hipStream_t st) {
    const int64_t n = (int64_t)ncell * ncell * ncell;
    const unsigned blocks = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(cell_dist_kernel, dim3(blocks), dim3(256), 0, st, occ, ncell, b, a, cap, 1);
    for (int it = 0; it < cap; ++it) {
        hipLaunchKernelGGL(cell_dist_kernel, dim3(blocks), dim3(256), 0, st, occ, ncell, a, b, cap, 0);
        uint8_t* t = a; a = b; b = t;
    }
    *result = a;
    return hipGetLastError();
}

hipError_t launch_occ_columns(const unsigned long long* occ, int ncell, unsigned long long* cols, hipStream_t st) {
    const int64_t n = 3 * (int64_t)ncell * ncell;
    hipLaunchKernelGGL(occ_columns_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, occ, ncell, cols);
    return hipGetLastError();
}

hipError_t launch_leaf_columns(const unsigned long long* locc, int nleaf, int cb_shift, unsigned long long* cols,
                               hipStream_t st) {
    const int64_t n = 3 * (int64_t)nleaf * nleaf;
    hipLaunchKernelGGL(leaf_columns_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, locc, nleaf, cb_shift,
                       cols);
    return hipGetLastError();
}

hipError_t launch_occupancy(const uint8_t* cls, const int32_t* maps, int nleaf, int cb_shift, int ncell,
                            const int64_t* lx, const int64_t* ly, const int64_t* lz, const uint8_t* alpha_nz,
                            int cls0, unsigned long long* occ, hipStream_t st) {
    const int64_t ncells = (int64_t)ncell * ncell * ncell;
    const int blocks = (int)std::min<int64_t>((ncells + 255) / 256, (int64_t)1 << 20);
    hipLaunchKernelGGL(occupancy_kernel, dim3(blocks), dim3(256), 0, st, cls, maps, nleaf, cb_shift, ncell,
                       lx, ly, lz, alpha_nz, cls0, occ);
    return hipGetLastError();
}


hipError_t launch_vrc_march(const VrcFrame& f, const WorkTile* work, const int32_t* order, int n_blocks,
                            const uint8_t* cls, const int32_t* maps, const int64_t* mapx64, const uint32_t* occ,
                            const float4* tf, int n_tf, float4* out, hipStream_t st, int batch, const float* vol,
                            const int32_t* rawmaps, const unsigned long long* occcol, const uint8_t* cdist,
                            const int32_t* gtab, int32_t* gtab_out, unsigned long long* count) {
    // (vrc_batch: K = 8 whenever empty cells are skipped, else 16).  count: the counting pass of
    // vr_count_marched (the same march, plus two atomics per ray into count[0..1])
    const bool k16 = vrc_batch(f, batch) == 16;
    if (count) {
        if (k16) launch_vrc_variant<2, 16>(f, work, order, n_blocks, cls, maps, mapx64, occ, tf, n_tf, out, count, st,
                                           vol, rawmaps, occcol, cdist, gtab, gtab_out);
        else launch_vrc_variant<2, 8>(f, work, order, n_blocks, cls, maps, mapx64, occ, tf, n_tf, out, count, st, vol,
                                      rawmaps, occcol, cdist, gtab, gtab_out);
    } else if (k16)
        launch_vrc_variant<0, 16>(f, work, order, n_blocks, cls, maps, mapx64, occ, tf, n_tf, out, nullptr, st,
                                  vol, rawmaps, occcol, cdist, gtab, gtab_out);
    else
        launch_vrc_variant<0, 8>(f, work, order, n_blocks, cls, maps, mapx64, occ, tf, n_tf, out, nullptr, st,
                                 vol, rawmaps, occcol, cdist, gtab, gtab_out);
    return hipGetLastError();
}

hipError_t launch_vrc_count(const VrcFrame& f, const WorkTile* work, int n_work, const int32_t* maps,
                            unsigned long long* total, hipStream_t st) {
    hipLaunchKernelGGL(vrc_count_kernel, dim3(n_work), dim3(kWgThreads), 0, st, f, work, maps, total);
    return hipGetLastError();
}

hipError_t launch_pack_classes(const uint8_t* c8, int64_t slots, int cbits, uint8_t* out, hipStream_t st) {
    const int64_t nbytes = (slots * cbits + 7) / 8;
    const int blocks = (int)std::min<int64_t>((nbytes + 255) / 256, 256 * 64);
    hipLaunchKernelGGL(pack_classes_kernel, dim3(blocks), dim3(256), 0, st, c8, slots, cbits, out);
    return hipGetLastError();
}

hipError_t launch_normals(const float* vol, int64_t d1, int64_t d2, int64_t d3, float4* nrm, hipStream_t st) {
    const int64_t n = d1 * d2 * d3;
    if (n == 0) return hipSuccess;
    const int64_t b64 = (n + 255) / 256;
    hipLaunchKernelGGL(normal_kernel, dim3((unsigned)(b64 < 65536 ? b64 : 65536)), dim3(256), 0, st, vol, d1, d2, d3,
                       nrm);
    return hipGetLastError();
}

hipError_t launch_assemble_list(int W, int H, int tile_w, int tile_h, const int32_t* slot_of, const float4* tiles,
                                float4 bg, float4* frame, int rgb, hipStream_t st, int n_frames) {
    const int64_t n = (int64_t)W * H;
    if (n == 0 || n_frames <= 0) return hipSuccess;
    const int nty = (H + tile_h - 1) / tile_h;
    const int64_t stride = (int64_t)((W + tile_w - 1) / tile_w) * nty;
    const dim3 grid((unsigned)((n + 255) / 256), (unsigned)n_frames);
    if (rgb)
        hipLaunchKernelGGL(assemble_list_kernel<true>, grid, dim3(256), 0, st, W, H, tile_w, tile_h, nty, slot_of, tiles,
                           bg, frame, stride);
    else
        hipLaunchKernelGGL(assemble_list_kernel<false>, grid, dim3(256), 0, st, W, H, tile_w, tile_h, nty, slot_of, tiles,
                           bg, frame, stride);
    return hipGetLastError();
}

hipError_t launch_assemble(int W, int H, int tile_w, int tile_h, int n_ranks, int max_tiles,
                           const float4* tiles, float4* frame, int rgb, hipStream_t st) {
    const int ntx = (W + tile_w - 1) / tile_w, nty = (H + tile_h - 1) / tile_h;
    const int64_t total = (int64_t)n_ranks * max_tiles * tile_w * tile_h;
    if (total == 0) return hipSuccess;
    if (rgb)
        hipLaunchKernelGGL(assemble_kernel<true>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, W, H, tile_w,
                           tile_h, ntx, nty, n_ranks, max_tiles, tiles, frame);
    else
        hipLaunchKernelGGL(assemble_kernel<false>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, W, H, tile_w,
                           tile_h, ntx, nty, n_ranks, max_tiles, tiles, frame);
    return hipGetLastError();
}

}  // namespace vr
