// vr_test.hip -- the TEST mode kernels (getColorFromNF + blendSampleColors, kernel.cu:72-187,
// :194-225) for gfx950: the general-view march over the corner-class volume, the plane-by-plane
// march of views along a volume axis, and their setup kernels (macro-cell occupancy, corner
// volume, per-line cell masks).  Split from vr_kernels.hip (VRC) so the two compile in parallel.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "vr_device.h"
#include "vr_march.h"

#pragma clang fp contract(off)

namespace vr {

// ------------------------------------------------------------------------------------------------
// TEST march: fused getColorFromNF + blendSampleColors (kernel.cu:72-187, :194-225).
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ void mulv3(const float* m, float x, float y, float z, float o[3]) {
    // glm mat4 * vec4(x, y, z, 1): (m0*x + m1*y) + (m2*z + m3*1), w dropped (vec3 truncation)
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        const float a0 = m[0 + r] * x + m[4 + r] * y;
        const float a1 = m[8 + r] * z + m[12 + r] * 1.0f;
        o[r] = a0 + a1;
    }
}

// a * (1 - w) + b * w (kernel.cu:162-175).  The exact (back-to-front) march evaluates it as written,
// every product and sum rounded (the contraction-off model of the whole restatement, oracle/), so
// exact TEST frames are bitwise the oracle's; the fast front-to-back march fuses the second product
// (a reassociation of the kind ERT already allows).
template <bool FUSED>
__device__ __forceinline__ float4 lerp4(float4 a, float4 b, float w) {
    const float u = 1.0f - w;
    // two channels per packed op: each half rounds like the scalar statement (unfused products and
    // sums stay unfused), so exact frames are unchanged bit for bit
    const f2 u2 = {u, u}, w2 = {w, w};
    const f2 axy = {a.x, a.y}, azw = {a.z, a.w}, bxy = {b.x, b.y}, bzw = {b.z, b.w};
    f2 lo, hi;
    if (FUSED) {
        lo = __builtin_elementwise_fma(bxy, w2, axy * u2);
        hi = __builtin_elementwise_fma(bzw, w2, azw * u2);
    } else {
        lo = axy * u2 + bxy * w2;
        hi = azw * u2 + bzw * w2;
    }
    return make_float4(lo.x, lo.y, hi.x, hi.y);
}

// Per sample (kernel.cu:100-115): p = T * (V * (Mcam * (x, y, s, 1))), three successive mat * vec.
// Inside iff 0 <= p_a < d_a (kernel.cu:92); corners c = p + {0,1}^3, flat index (int)c.x*d2*d3 +
// (int)c.y*d3 + (int)c.z with only the idx < total guard (a corner at c.z == d3 wraps to the next
// row, like the reference); each corner classified TF(v / cal_max) (the TEST class volume); RGBA
// lerped in y, then x, then z (kernel.cu:162-175).  Outside -> TF(0).
//
// Batched like the VRC march: K samples' positions and 8K class gathers are issued before any is
// used, then composited in order.  ESS skips macro cells of 2^tcb voxels (+2-voxel apron, since
// (int)(p + 1) can reach floor(p) + 2) whose classes are all alpha 0; cells at an upper face, where
// corner indices wrap, are always occupied.  Jumps use the linear model p(s) ~ pa + s*dp with a
// 0.05-voxel safety margin, so every skipped sample lies inside the empty cell.
//
// Whole TEST frames: work tiles off the dataset box's projection (vr_api.cpp project_box_test) are
// exactly the background; a background-only workgroup (blockIdx >= bg_first) stores bg_group of
// them, and a culled tile (slot < 0) among the marching ones stores its own -- both before any
// staging.  True if this workgroup is done.
__device__ __forceinline__ bool test_background(const TestFrame& f, const WorkTile* __restrict__ work, const WorkTile& wt,
                                                float4* __restrict__ out) {
    if (f.out_tiles) return false;
    const float4 bg = make_float4(f.bg[0], f.bg[1], f.bg[2], 1.0f);
    if ((int)blockIdx.x >= f.bg_first) {
        const int e0 = f.bg_first + ((int)blockIdx.x - f.bg_first) * f.bg_group;
        for (int i = 0; i < f.bg_group; ++i) {
            const int e = e0 + i;
            if (e >= f.n_work) break;
            int x, y;
            ray_of_thread(work[e], x, y);
            if (x < f.W && y < f.H) store_f4(out + (int64_t)x * f.H + y, bg);
        }
        return true;
    }
    bool off = wt.slot < 0;
    // general views: a work tile inside the visible rectangle but off the projected box's hull
    // (separated by one of its edges, vr_api.cpp hull_edges) sees only TF(0): the background too.
    // Wave-uniform: the tile's pixels [x0, x0 + 16) x [y0, y0 + 16) against each edge's half-plane.
    // (unrolled over kMaxHull so the edges' kernel-argument loads issue together)
#pragma unroll
    for (int e = 0; e < kMaxHull; ++e) {
        const float nx = f.hull[e][0], ny = f.hull[e][1];
        const float px = (float)wt.x0 + (nx > 0.0f ? 0.0f : (float)(kWgRaysX - 1));
        const float py = (float)wt.y0 + (ny > 0.0f ? 0.0f : (float)(kWgRaysY - 1));
        off |= (e < f.n_hull) & (nx * px + ny * py > f.hull[e][2]);   // (bitwise: no branch per edge)
    }
    if (!off) return false;
    int x, y;
    ray_of_thread(wt, x, y);
    if (x < f.W && y < f.H) store_f4(out + (int64_t)x * f.H + y, bg);
    return true;
}

// CV = the corner volume a sample's 8 corner classes come from in ONE gather (host: class 0 = TF(0),
// 32-bit offsets): 0 none (four corner-row dwords of the class volume); CB = 2 / 4 / 8 bits per
// corner class (the TF's class width: 16 / 32 / 64 bits, i.e. CB bytes, per voxel) either in the
// reference's x-major voxel order (CV = 16 + CB: byte offset CB * flat index, the flat index's own
// arithmetic) or in 4 x 4 x 4-voxel bricks (CV = CB: voxel (x, y, z) at byte offset lay[x] +
// lay[d1 + y] + lay[d1 + d2 + z], separable tables staged in LDS).  STATS 2: the counting pass of
// vr_count_work (gathers, bytes, samples evaluated into stats[0..2]).
template <int CV> struct CornerBits { static constexpr int value = CV == 0 ? 8 : (CV & 15); };

// Field of corner kk = (x << 2 | y << 1 | z) in a corner-volume entry: the z = 0 plane's corners first,
// (x, y) at 2x + y, then the z = 1 plane's -- so with 2-bit classes each plane's 4 classes are one
// byte, the index of its row of the plane table (PT below).  Bits [CB f, CB f + CB) of the entry.
__host__ __device__ constexpr int corner_field(int kk) { return ((kk & 1) << 2) | (kk >> 1); }

// PT (front to back, 2-bit classes, i.e. TFs of at most 4 intervals): the plane table.  A z-plane of
// a sample's corners is one byte key = c00 | c01 << 2 | c10 << 4 | c11 << 6 (c_xy its 2-bit classes);
// its y-then-x lerp (kernel.cu:162-169) in fused form is T0 + wy T1 + wx T2 + wx wy T3 with
//   T0 = col(c00), T1 = col(c01) - col(c00), T2 = col(c10) - col(c00), T3 = col(c11) - col(c10) - T1,
// 256 keys x 4 float4 = 16 KB of LDS, component-major (row i at 16 (256 i + key): the lanes' distinct
// keys fall in distinct bank slots mod 16).  Built per workgroup from the TF.  A sample is then
// 8 ds_read_b128 + 7 packed fma and no class extraction, against 8 class extractions, 8 TF reads and
// 7 four-wide lerps; all-equal corners need no special case (T1 = T2 = T3 = 0).  The exact
// (back-to-front) march keeps the reference's lerps.
constexpr int kPtKeys = 256;
constexpr size_t kPtBytes = 4 * kPtKeys * 16;
static_assert(kPtKeys == kWgThreads, "the plane table is built one key per thread");

#ifndef VR_TEST_WAVES
#define VR_TEST_WAVES 1
#endif
template <bool F2B, bool ESS, bool IDX64, int K, bool SEP, int CV, bool PT, int STATS = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(PT ? VR_TEST_WAVES : 1))) void test_march_kernel(TestFrame f, const WorkTile* __restrict__ work,
                                                         const int32_t* __restrict__ order,
                                                         const uint8_t* __restrict__ cls,
                                                         const float4* __restrict__ tf_rgba, int n_tf,
                                                         const uint32_t* __restrict__ gocc,
                                                         float4* __restrict__ out,
                                                         const uint8_t* __restrict__ cvol,
                                                         const int32_t* __restrict__ clay,
                                                         unsigned long long* __restrict__ stats) {
    using idx_t = typename IdxT<IDX64>::type;
    constexpr bool CORN = CV != 0;                  // one gather per sample from a corner volume
    constexpr bool BRICK = CV != 0 && CV < 16;      // ... in 4^3-voxel bricks
    constexpr int CB = CornerBits<CV>::value;       // bits per corner class
    constexpr uint32_t CMASK = (1u << CB) - 1u;
    constexpr bool PTX = PT && F2B && CORN && CB == 2;   // the plane table (above)
// (VR_TEST_LIN: off -- see march_pos below and DESIGN "Round 6")
#ifndef VR_TEST_LIN
#define VR_TEST_LIN 0
#endif
    constexpr bool LIN = VR_TEST_LIN && PTX && SEP;      // linear-model positions (below)
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_all[];
    float4* s_pt = reinterpret_cast<float4*>(smem_all);
    unsigned char* smem = smem_all + (PTX ? kPtBytes : 0);
    float4* s_tf = reinterpret_cast<float4*>(smem);
    uint32_t* s_occ = reinterpret_cast<uint32_t*>(smem + (size_t)n_tf * sizeof(float4));
    // SEP: the per-sample half of the second product, B_r(s) = iv_{8+r} q1z(s) + iv_{12+r} with
    // q1z(s) = mc10 s + mc14, is the same for every ray: a per-frame table, (B_0, B_1, B_2, 0) at
    // s_B[s + K] for s in [-K, S + K) (one ds_read_b128 per sample instead of eight VALU operations)
    float4* s_B = reinterpret_cast<float4*>(smem + (size_t)n_tf * sizeof(float4) +
                                            (((ESS && f.occ_lds) ? (size_t)f.occ_words * 4 : 0) + 15) / 16 * 16);
    // BRICK: the corner volume's separable offset tables (d1 + d2 + d3 int32) after the B table
    int32_t* s_lay = reinterpret_cast<int32_t*>(s_B + ((SEP && f.sep_tab) ? f.S + 2 * K : 0));
    const int nlay = (int)(f.d1 + f.d2 + f.d3);
    // The first round of loads -- the TF entry, up to 4 occupancy words and brick-table entries per
    // lane, and the work tile -- is issued together; a culled work tile (or a background-only
    // workgroup) then stores the background and leaves before any LDS staging (the loads it issued
    // are independent of the tile, so a marching workgroup's prologue waits for one round only).
    const bool occ_st = ESS && f.occ_lds;
    // (unconditional, index clamped; stored only for threadIdx.x < n_tf <= kMaxTf = kWgThreads, host)
    const float4 tfv = tf_rgba[(int)threadIdx.x < n_tf ? (int)threadIdx.x : 0];
    // PT: this thread's key's 4 classified colours (classes past the TF clamped: never marched)
    float4 ptc[4];
    if (PTX) {
#pragma unroll
        for (int i = 0; i < 4; ++i) ptc[i] = tf_rgba[min(((int)threadIdx.x >> (2 * i)) & 3, n_tf - 1)];
    }
    // the frame constants the exits branch on, loaded in the first round (vrc_march_kernel)
    asm volatile("" ::"s"(f.out_tiles), "s"(f.bg_first), "s"(f.n_work), "s"(f.n_hull), "s"(f.W), "s"(f.H));
    uint32_t ov[4];
    int32_t lv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int i = (int)threadIdx.x + u * kWgThreads;
        // unconditional loads (index clamped, value selected): a load under its range test is
        // waited for inside the branch, one round trip per entry
        const bool io = occ_st && i < f.occ_words;
        ov[u] = 0u;
        if (ESS) { const uint32_t w = gocc[io ? i : 0]; ov[u] = io ? w : 0u; }
        lv[u] = 0;
        if (BRICK) { const int32_t w = clay[i < nlay ? i : 0]; lv[u] = i < nlay ? w : 0; }
    }
    // (the work tile load is unconditional: guarded, each kernel argument of the guard would be
    // loaded and waited for in turn before it issues; `order` is unused -- every caller passes null)
    const int b = (int)blockIdx.x;
    const WorkTile wt = work[b < f.n_work ? b : 0];
    if (b >= f.n_work) return;
    if (test_background(f, work, wt, out)) return;
    if ((int)threadIdx.x < n_tf) s_tf[threadIdx.x] = tfv;
    if (PTX) {
        auto sub = [](float4 a, float4 b) { return make_float4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w); };
        const float4 t1 = sub(ptc[1], ptc[0]);
        s_pt[threadIdx.x] = ptc[0];
        s_pt[kPtKeys + threadIdx.x] = t1;
        s_pt[2 * kPtKeys + threadIdx.x] = sub(ptc[2], ptc[0]);
        s_pt[3 * kPtKeys + threadIdx.x] = sub(sub(ptc[3], ptc[2]), t1);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int i = (int)threadIdx.x + u * kWgThreads;
        if (occ_st && i < f.occ_words) s_occ[i] = ov[u];
        if (BRICK && i < nlay) s_lay[i] = lv[u];
    }
    if (occ_st)
        for (int i = threadIdx.x + 4 * kWgThreads; i < f.occ_words; i += kWgThreads) s_occ[i] = gocc[i];
    if (BRICK)
        for (int i = threadIdx.x + 4 * kWgThreads; i < nlay; i += kWgThreads) s_lay[i] = clay[i];
    if (SEP && f.sep_tab && !(LIN && f.lin))
        for (int j = threadIdx.x; j < f.S + 2 * K; j += kWgThreads) {
            const float q1z = f.mc[10] * (float)(j - K) + f.mc[14];
            s_B[j] = make_float4(f.iv[8] * q1z + f.iv[12] * 1.0f, f.iv[9] * q1z + f.iv[13] * 1.0f,
                                 f.iv[10] * q1z + f.iv[14] * 1.0f, 0.0f);
        }
    __syncthreads();
    // the occupancy word of a cell: from LDS through ds_read, else through a buffer load -- one
    // pointer chosen at run time compiled to a flat load that waited on both counters every batch
    const __amdgpu_buffer_rsrc_t ors = uniform_rsrc(gocc, ESS ? f.occ_words * 4 : 0);
    auto occ_word = [&](int wi) -> uint32_t {
        if (f.occ_lds) return s_occ[wi];
        return __builtin_amdgcn_raw_buffer_load_b32(ors, wi * 4, 0, 0);
    };
    // the ERT threshold in a VGPR: reloaded from the kernel arguments every batch, its s_load's
    // lgkmcnt(0) also waited for the batch's LDS reads (vrc_march_kernel)
    float ert_eps = f.ert_eps;
    asm volatile("" : "+v"(ert_eps));
    int x, y;
    ray_of_thread(wt, x, y);
    if (x >= f.W || y >= f.H) return;

    const float fx = (float)x, fy = (float)y;
    // first product, split: Add0 = m0*x + m1*y per ray; Add1 = m2*s + m3 per sample
    float add0[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) add0[r] = f.mc[0 + r] * fx + f.mc[4 + r] * fy;
    // SEP (always, for the matrices kernel.cu:1177-1216 builds: modelCam and toVolume are scales +
    // translations): the zero entries of mc and tv contribute exact zeros to glm's
    // (m0*x + m1*y) + (m2*z + m3) (x + 0 = x, and a zero's sign cannot reach a frame value), so
    // q1 = (mc0*x + mc12, mc5*y + mc13, mc10*s + mc14) and p_r = tv_rr * q2_r + tv_3r bit for bit.
    // inverse(lookAt) is general, but its first pair iv_r*q1x + iv_4+r*q1y only depends on the
    // ray: per sample 17 operations instead of 51, the same roundings in the same order.
    float A[3];
    if (SEP) {
        const float q1x = f.mc[0] * fx + f.mc[12], q1y = f.mc[5] * fy + f.mc[13];
#pragma unroll
        for (int r = 0; r < 3; ++r) A[r] = f.iv[r] * q1x + f.iv[4 + r] * q1y;
    }

    auto position = [&](int s, float p[3]) {
        const float fs = (float)s;
        if (SEP) {
            // (s in [-K, S + K): the batches' samples, valid or not, and the clip's ends).  Without
            // the table (long rays: it would not fit LDS) the same expressions per sample.
            float4 Bs;
            if (f.sep_tab && !(LIN && f.lin)) {   // (linear positions: no table -- only the ray's end points come here)
                Bs = s_B[s + K];
            } else {
                const float q1z = f.mc[10] * fs + f.mc[14];
                Bs = make_float4(f.iv[8] * q1z + f.iv[12] * 1.0f, f.iv[9] * q1z + f.iv[13] * 1.0f,
                                 f.iv[10] * q1z + f.iv[14] * 1.0f, 0.0f);
            }
            float q2[3];
            q2[0] = A[0] + Bs.x;
            q2[1] = A[1] + Bs.y;
            q2[2] = A[2] + Bs.z;
            p[0] = f.tv[0] * q2[0] + f.tv[12];
            p[1] = f.tv[5] * q2[1] + f.tv[13];
            p[2] = f.tv[10] * q2[2] + f.tv[14];
            return;
        }
        float q1[3], q2[3];
#pragma unroll
        for (int r = 0; r < 3; ++r) q1[r] = add0[r] + (f.mc[8 + r] * fs + f.mc[12 + r] * 1.0f);
        mulv3(f.iv, q1[0], q1[1], q1[2], q2);
        mulv3(f.tv, q2[0], q2[1], q2[2], p);
    };

    // The ray's linear model p(s) ~= pa + s dp (from its exact end points) and its conservative clip
    // to the volume widened by 0.01 voxel: samples outside [s_begin, s_end) are outside the volume,
    // TF(0), alpha 0 (zero_transparent).  In float: p(s) itself departs from the line by a few ulps of
    // |p| (~1e-5 voxel), the float quotients by ~1e-7 of s (< 1e-3 samples at S = 9k) -- far inside
    // the 0.01-voxel and floor - 1 / ceil + 2 margins.  (Round 4 did this in double: ~150 FP64
    // instructions per wave, half-rate, for the same range.)  A zero step tests the point; a
    // denormal one gives an infinite reciprocal, whose products keep the test conservative (a NaN
    // from 0 * inf is ignored by fminf / fmaxf: no constraint).
    int s_begin = 0, s_end = f.S;
    float pa[3], dp[3], idp[3];
    {
        float pb[3];
        position(0, pa);
        position(f.S > 1 ? f.S - 1 : 0, pb);
        const float dims[3] = {f.fd1, f.fd2, f.fd3};
        const float den = (float)(f.S > 1 ? f.S - 1 : 1);
        float a = 0.0f, bnd = (float)(f.S - 1);
        bool off = false;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            dp[c] = f.S > 1 ? (pb[c] - pa[c]) / den : 0.0f;
            idp[c] = dp[c] != 0.0f ? 1.0f / dp[c] : 0.0f;
            const float lo = -0.01f, hi = dims[c] + 0.01f;
            if (dp[c] == 0.0f) {
                off |= (pa[c] < lo) | (pa[c] > hi);
            } else {
                const float t0 = (lo - pa[c]) * idp[c], t1 = (hi - pa[c]) * idp[c];
                a = fmaxf(a, fminf(t0, t1));
                bnd = fminf(bnd, fmaxf(t0, t1));
            }
        }
        if (f.zero_transparent) {
            if (off || !(a <= bnd)) {
                s_end = 0;
            } else {
                s_begin = max(0, (int)floorf(a) - 1);
                s_end = min(f.S, (int)ceilf(bnd) + 2);
            }
        }
    }

    // LIN (the plane table's front-to-back march, within the ERT tolerance): a sample's position from
    // the ray's linear model, p = pa + s dp (3 fmas), instead of the reference's chain through the
    // per-sample table s_B (an LDS read in every sample's dependency chain, then 9 operations).  The
    // model departs from the chain by a few ulps of |p| (~2e-5 voxel at the MNI shape); trilinear
    // interpolation is continuous, so a sample's colour moves by at most that times the colour step
    // between neighbouring voxels (<= 1): <= 2e-5 per sample, inside the 1e-4 of the ERT frames.  The
    // corner choice, the p + 1 test, the cell of the empty-cell test and the clip all follow the same
    // p, so they stay consistent with each other.  Only when every voxel on the volume's six faces is
    // class 0 (f.lin, host: test_faces_kernel): the colour is then continuous across the faces too
    // (TF(0) on both sides); otherwise a sample within a few ulps of a face could take the other side
    // of the reference's in-volume test, a jump of up to a whole colour.
    auto march_pos = [&](int sk, float p[3]) {
        if (LIN && f.lin) {
            const float fs = (float)sk;
#pragma unroll
            for (int c = 0; c < 3; ++c) p[c] = fmaf(fs, dp[c], pa[c]);
        } else {
            position(sk, p);
        }
    };

    const float4 tf0 = s_tf[f.cls0];
    const idx_t d3 = (idx_t)f.d3, d23 = (idx_t)(f.d2 * f.d3), total = (idx_t)f.total;
    const __amdgpu_buffer_rsrc_t trs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(cls), (short)0, IDX64 ? 0 : (int)f.total + kClsPad / 4,
                                          0x00020000);
    float r, g, bl, T = 1.0f;
    if (F2B) { r = 0.0f; g = 0.0f; bl = 0.0f; }
    else { r = f.bg[0]; g = f.bg[1]; bl = f.bg[2]; }

    unsigned st_g = 0, st_b = 0, st_it = 0;   // STATS: gathers, bytes, samples evaluated
    int s = F2B ? s_begin : s_end - 1;
    bool done = F2B ? (s >= s_end) : (s < s_begin);
    float pfirst[3];   // ESS: the position of the batch's first sample, from the empty-cell test
#ifndef VR_TEST_LAZY
#define VR_TEST_LAZY 0
#endif
    // LAZY (front to back): the empty-cell test only after a batch that composited nothing (T
    // unchanged); inside tissue its position, cell and occupancy read are skipped
    constexpr bool LAZY = VR_TEST_LAZY && ESS && F2B;
    bool ess_check = true;
    while (!done) {
        const float T_batch = T;
        if (ESS && !LAZY) march_pos(s, pfirst);
        if (ESS && (!LAZY || ess_check)) {
            float* p = pfirst;
            if (LAZY) march_pos(s, p);
            // (bitwise, not short-circuit: && chains compile to exec-mask branches, SALU per sample)
            const bool inside = ((int)(__float_as_uint(p[0]) < __float_as_uint(f.fd1)) &
                                 (int)(__float_as_uint(p[1]) < __float_as_uint(f.fd2)) &
                                 (int)(__float_as_uint(p[2]) < __float_as_uint(f.fd3))) != 0;
            int cc[3];
#pragma unroll
            for (int c = 0; c < 3; ++c) cc[c] = inside ? ((int)p[c] >> f.tcb) : 0;
            const int cell = __mul24(__mul24(cc[0], f.tnc[1]) + cc[1], f.tnc[2]) + cc[2];   // (< 2^18 cells)
            if (inside && !((occ_word(cell >> 5) >> (cell & 31)) & 1u)) {
                float sstar = F2B ? 3.0e38f : -3.0e38f;
                const float B = (float)(1 << f.tcb);
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    if (dp[c] == 0.0f) continue;
                    const bool up_axis = F2B ? (dp[c] > 0.0f) : (dp[c] < 0.0f);
                    const float bound = up_axis ? (float)(cc[c] + 1) * B - 0.05f : (float)cc[c] * B + 0.05f;
                    const float sc = (bound - pa[c]) * idp[c];   // (the 0.05-voxel margin covers the rounding)
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
        if (STATS) st_it += K;
        float w[K][3];
        bool in[K];
        int cl[K][8];
        // CORN (host: class 0 = TF(0), 32-bit offsets, the corner volume built): a sample's 8 corner
        // classes are ONE gather from the corner volume (test_corner_kernel: voxel idx holds the
        // classes at flat idx + {0, 1, d3, d3 + 1, d2 d3, ...}, the reference's flat-index wrap and
        // idx < total guard built in) -- whenever every (int)(p + 1) is (int)p + 1.  A sample whose
        // p + 1 rounds up to (int)p + 2 on some axis (p within half an ulp of the next integer) takes
        // the dword gathers below instead, exec-masked, packed like the corner volume.  Corner kk =
        // (x << 2 | y << 1 | z) sits at bit CB corner_field(kk) of (clo, chi).
        uint32_t clo[K], chi[K];
        int coff[K];
        // class 0 = TF(0 / cal_max) (the usual TF) and 32-bit indices: the corner gathers go through a
        // buffer resource bounded at `total`, which IS the reference's idx < total guard (an index at
        // or past the end reads class 0 = cls0); samples outside the volume get an out-of-range
        // offset.  No idx < total compares and no 64-bit address arithmetic; the loads stay
        // exec-masked per sample, so lanes outside the volume skip them (the masked form measured
        // best: unmasked or wave-uniform skips cost the oblique camera 10 %).
        const bool buf = !IDX64 && f.cls0 == 0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int sk = F2B ? s + k : s - k;
            const bool valid = F2B ? (sk < s_end) : (sk >= s_begin);
            float p[3];
            if (ESS && !LAZY && k == 0) {   // (s did not move since the empty-cell test: the same position)
                p[0] = pfirst[0]; p[1] = pfirst[1]; p[2] = pfirst[2];
            } else {
                march_pos(sk, p);
            }
            // 0 <= p < fd as unsigned compares of the bits (fd > 0; NaN and negatives compare high;
            // p is never -0: its last term tv[12+r] = d_r / 2 is not 0, and an exact cancellation
            // rounds to +0)
            in[k] = ((int)valid & (int)(__float_as_uint(p[0]) < __float_as_uint(f.fd1)) &
                     (int)(__float_as_uint(p[1]) < __float_as_uint(f.fd2)) &
                     (int)(__float_as_uint(p[2]) < __float_as_uint(f.fd3))) != 0;
            idx_t i0[3], i1[3];
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                i0[c] = (idx_t)(int)p[c];
                i1[c] = CORN ? 0 : (idx_t)(int)(p[c] + 1.0f);   // (CORN: below, when needed)
                // p - (float)(int)p: for an in-volume sample (p >= 0) that is p - floor(p), which
                // v_fract_f32 returns exactly (the difference is representable); outside, unused
                w[k][c] = __builtin_amdgcn_fractf(p[c]);
            }
            if (CORN) {
                // (int)(p + 1) == (int)p + 1 on every axis (one gather from the corner volume).  p + 1 =
                // n + 1 + f exactly (n = (int)p, f its fraction) rounds up to n + 2 only when 1 - f <=
                // ulp(n + 2) / 2 <= ulp(d + 1) / 2, so f below 1 - ulp(d + 1) (wthr, host) settles it
                // with one compare per axis; the integer test runs only past that bound (~2^-15 of
                // samples per axis at the MNI shape)
                bool d111 = ((int)(w[k][0] < f.wthr[0]) & (int)(w[k][1] < f.wthr[1]) & (int)(w[k][2] < f.wthr[2])) != 0;
                if (in[k] && !d111) {
#pragma unroll
                    for (int c = 0; c < 3; ++c) i1[c] = (idx_t)(int)(p[c] + 1.0f);
                    d111 = ((int)((i1[0] - i0[0]) == 1) & (int)((i1[1] - i0[1]) == 1) & (int)((i1[2] - i0[2]) == 1)) != 0;
                }
                int o;
                if (BRICK) {   // separable brick offsets (indices clamped: only in-volume samples use them)
                    o = s_lay[min((unsigned)i0[0], (unsigned)f.d1 - 1u)] +
                        s_lay[(int)f.d1 + (int)min((unsigned)i0[1], (unsigned)f.d2 - 1u)] +
                        s_lay[(int)(f.d1 + f.d2) + (int)min((unsigned)i0[2], (unsigned)f.d3 - 1u)];
                } else {
                    // (CB bits x 8 corners = CB bytes); 24-bit multiplies (full rate: v_mul_lo_u32 issues
                    // at a quarter of it) -- a corner volume is used only when d1 and d2 d3 are below
                    // 2^24 (host: launch_test_march)
                    o = (int)(__umul24((unsigned)i0[0], (unsigned)d23) + __umul24((unsigned)i0[1], (unsigned)d3) +
                              (unsigned)i0[2]) * CB;
                }
                coff[k] = (in[k] && d111) ? o : 0x7ffffff0;
                clo[k] = 0u; chi[k] = 0u;
                if (STATS) { st_g += in[k] && d111; st_b += (in[k] && d111) ? CB : 0u; }
                if (in[k] && !d111) {   // (rare) the corner rows' dwords, packed like the corner volume
                    const unsigned zb = (unsigned)(i1[2] - i0[2]) * 8u;
#pragma unroll
                    for (int xy = 0; xy < 4; ++xy) {
                        const idx_t rx = (xy >> 1) & 1 ? i1[0] : i0[0], ry = xy & 1 ? i1[1] : i0[1];
                        // (24-bit multiplies as above: a 32-bit one here was hoisted onto every sample)
                        const int ri = (int)(__umul24((unsigned)rx, (unsigned)d23) + __umul24((unsigned)ry, (unsigned)d3) +
                                             (unsigned)i0[2]);
                        const uint32_t wd = __builtin_amdgcn_raw_buffer_load_b32(trs, ri, 0, 0);
                        // corners 2xy (z0: field xy) and 2xy + 1 (z1: field 4 + xy)
                        const uint32_t z0 = wd & 0xffu, z1 = (wd >> zb) & 0xffu;
                        if (CB < 8) {
                            clo[k] |= (z0 << (CB * xy)) | (z1 << (CB * (4 + xy)));
                        } else {
                            clo[k] |= z0 << (8 * xy);
                            chi[k] |= z1 << (8 * xy);
                        }
                    }
                    if (STATS) { st_g += 4; st_b += 16; }
                }
            } else if (buf) {
                // the two z corners of an (x, y) corner row are flat indices idx and idx + dz (dz =
                // (int)(p_z + 1) - (int)p_z, 1 or 2): one unaligned dword at idx holds both bytes, with
                // the flat-index wrap of the reference intact.  Offsets for now; loaded below.
#pragma unroll
                for (int xy = 0; xy < 4; ++xy) {
                    const int idx = (int)(((xy >> 1) & 1 ? i1[0] : i0[0]) * d23 + (xy & 1 ? i1[1] : i0[1]) * d3 + i0[2]);
                    cl[k][2 * xy] = in[k] ? idx : 0x7fffffff;
                }
                cl[k][1] = (int)(i1[2] - i0[2]) * 8;   // bit offset of the upper z corner
                if (STATS) { st_g += in[k] ? 4u : 0u; st_b += in[k] ? 16u : 0u; }
            } else {
#pragma unroll
                for (int kk = 0; kk < 8; ++kk) {
                    const idx_t idx = ((kk >> 2) & 1 ? i1[0] : i0[0]) * d23 + ((kk >> 1) & 1 ? i1[1] : i0[1]) * d3 +
                                      (kk & 1 ? i1[2] : i0[2]);
                    cl[k][kk] = (in[k] && idx < total) ? (int)cls[idx] : f.cls0;
                    if (STATS) { st_g += in[k] && idx < total; st_b += in[k] && idx < total; }
                }
            }
        }
        if (CORN) {
            const __amdgpu_buffer_rsrc_t crs = uniform_rsrc(cvol, f.cv_bytes);
#pragma unroll
            for (int k = 0; k < K; ++k) {   // (out of range: 0)
                if (CB == 8) {
                    const auto v = __builtin_amdgcn_raw_buffer_load_b64(crs, coff[k], 0, 0);
                    clo[k] |= v[0];
                    chi[k] |= v[1];
                } else if (CB == 4) {
                    clo[k] |= __builtin_amdgcn_raw_buffer_load_b32(crs, coff[k], 0, 0);
                } else {
                    clo[k] |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(crs, coff[k], 0, 0);
                }
            }
        } else if (buf) {
#pragma unroll
            for (int k = 0; k < K; ++k) {
                if (in[k]) {   // exec-masked: lanes outside skip the gathers
                    const int zb = cl[k][1];
                    uint32_t wd[4];
#pragma unroll
                    for (int xy = 0; xy < 4; ++xy) wd[xy] = __builtin_amdgcn_raw_buffer_load_b32(trs, cl[k][2 * xy], 0, 0);
#pragma unroll
                    for (int xy = 0; xy < 4; ++xy) {
                        cl[k][2 * xy] = (int)(wd[xy] & 0xffu);
                        cl[k][2 * xy + 1] = (int)((wd[xy] >> zb) & 0xffu);
                    }
                } else {
#pragma unroll
                    for (int kk = 0; kk < 8; ++kk) cl[k][kk] = 0;
                }
            }
        }
        // a batch in which every lane's samples are outside or between class-0 corners (class 0 =
        // TF(0), alpha 0) composites nothing: f * (1 - 0) + c * 0 = f and T * (1 - 0) = T, bit for
        // bit.  The whole wave skips its TF reads and lerps (a wave-uniform branch).
        bool blank = buf && f.zero_transparent;
        if (blank) {
            bool mine = true;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                if (CORN) {
                    mine = mine && (clo[k] | chi[k]) == 0u;
                } else {
#pragma unroll
                    for (int kk = 0; kk < 8; ++kk) mine = mine && cl[k][kk] == 0;
                }
            }
            blank = __all(mine);
        }
        if (!blank) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            float4 cf = tf0;
            if (PTX) {
                // the plane table: z0 plane = entry bits 0-7, z1 plane = bits 8-15 (corner_field);
                // outside the volume the value is replaced by TF(0) (no branch: the gathers of
                // those lanes returned 0 anyway)
                const uint32_t k0 = clo[k] & 0xffu, k1 = (clo[k] >> 8) & 0xffu;
                const float dx = w[k][0], dy = w[k][1], dz = w[k][2], dxy = dx * dy;
                const f2 X = {dx, dx}, Y = {dy, dy}, XY = {dxy, dxy}, Z = {dz, dz};
                auto plane = [&](uint32_t key, f2& lo, f2& hi) {
                    const float4 a0 = s_pt[key], a1 = s_pt[kPtKeys + key];
                    const float4 a2 = s_pt[2 * kPtKeys + key], a3 = s_pt[3 * kPtKeys + key];
                    lo = __builtin_elementwise_fma(
                        XY, f2{a3.x, a3.y},
                        __builtin_elementwise_fma(X, f2{a2.x, a2.y}, __builtin_elementwise_fma(Y, f2{a1.x, a1.y}, f2{a0.x, a0.y})));
                    hi = __builtin_elementwise_fma(
                        XY, f2{a3.z, a3.w},
                        __builtin_elementwise_fma(X, f2{a2.z, a2.w}, __builtin_elementwise_fma(Y, f2{a1.z, a1.w}, f2{a0.z, a0.w})));
                };
#ifndef VR_PT_UNI
#define VR_PT_UNI 0
#endif
#ifndef VR_PT_SELECT
#define VR_PT_SELECT 0
#endif
                // every lane's 8 corners of one class (or the sample outside): the table's value is
                // that class's colour exactly (T1 = T2 = T3 = 0: each fma adds an exact zero), one TF
                // read -- a wave-uniform branch, taken by whole waves inside homogeneous tissue
                const bool uni8 = clo[k] == (clo[k] & 3u) * 0x5555u;
                if (VR_PT_UNI && __all(uni8 || !in[k])) {
                    cf = in[k] ? s_tf[clo[k] & 3u] : tf0;
                } else {
                    f2 p0l, p0h, p1l, p1h;
                    plane(k0, p0l, p0h);
                    plane(k1, p1l, p1h);
                    const f2 lo = __builtin_elementwise_fma(Z, p1l - p0l, p0l), hi = __builtin_elementwise_fma(Z, p1h - p0h, p0h);
                    if (VR_PT_SELECT) {
                        // (bit select: no exec-mask branch around the table reads)
                        const unsigned m = in[k] ? 0xffffffffu : 0u;
                        auto sel = [&](float a, float b) {
                            return __uint_as_float((__float_as_uint(a) & m) | (__float_as_uint(b) & ~m));
                        };
                        cf = make_float4(sel(lo.x, tf0.x), sel(lo.y, tf0.y), sel(hi.x, tf0.z), sel(hi.y, tf0.w));
                    } else {
                        cf = in[k] ? make_float4(lo.x, lo.y, hi.x, hi.y) : tf0;
                    }
                }
            }
            // front to back (ERT, fused lerps): a sample whose 8 corner classes are equal is that
            // class's colour -- the lerps of equal colours, within the fused form's rounding (<= 2
            // ulp, inside the ERT tolerance): one TF read, no lerps.  Exact mode keeps every lerp.
            bool uni = false;
            if (F2B && !PTX) {
                if (CORN) {
                    // the 8 fields all equal the first: its value times the field-replication constant
                    constexpr uint32_t rep = CB == 2 ? 0x5555u : (CB == 4 ? 0x11111111u : 0x01010101u);
                    uni = (CB < 8 || clo[k] == chi[k]) && clo[k] == (clo[k] & CMASK) * rep;
                } else {
                    uni = true;
#pragma unroll
                    for (int kk = 1; kk < 8; ++kk) uni = uni && cl[k][kk] == cl[k][0];
                }
            }
            if (PTX) {
                // (above)
            } else if (F2B && in[k] && uni) {
                cf = s_tf[CORN ? (int)(clo[k] & CMASK) : cl[k][0]];
            } else if (in[k]) {
                if (CORN) {
#pragma unroll
                    for (int kk = 0; kk < 8; ++kk) {
                        const int fk = corner_field(kk);   // (CB 8: z0 plane in clo, z1 in chi)
                        cl[k][kk] = CB == 8 ? (int)(((fk < 4 ? clo[k] : chi[k]) >> (8 * (fk & 3))) & 0xffu)
                                            : (int)((clo[k] >> (CB * fk)) & CMASK);
                    }
                }
                float4 cc[8];
#pragma unroll
                for (int kk = 0; kk < 8; ++kk) cc[kk] = s_tf[cl[k][kk]];
                const float dx = w[k][0], dy = w[k][1], dz = w[k][2];
                const float4 y1 = lerp4<F2B>(cc[0], cc[2], dy), y2 = lerp4<F2B>(cc[1], cc[3], dy);
                const float4 y3 = lerp4<F2B>(cc[4], cc[6], dy), y4 = lerp4<F2B>(cc[5], cc[7], dy);
                const float4 z1 = lerp4<F2B>(y1, y3, dx), z2 = lerp4<F2B>(y2, y4, dx);
                cf = lerp4<F2B>(z1, z2, dz);
            }
            const int sk = F2B ? s + k : s - k;
            const float a = (F2B ? (sk < s_end) : (sk >= s_begin)) ? cf.w : 0.0f;
            if (F2B) {
                const float wt_ = T * a;
                r = fmaf(wt_, cf.x, r); g = fmaf(wt_, cf.y, g); bl = fmaf(wt_, cf.z, bl);
                T = T * (1.0f - a);
            } else {
                r = r * (1 - a) + cf.x * a;
                g = g * (1 - a) + cf.y * a;
                bl = bl * (1 - a) + cf.z * a;
            }
        }
        }   // !blank
        if (LAZY) ess_check = T == T_batch;
        if (F2B && T < ert_eps) done = true;
        s = F2B ? s + K : s - K;
        if (F2B ? (s >= s_end) : (s < s_begin)) done = true;
    }
    if (F2B) { r = r + T * f.bg[0]; g = g + T * f.bg[1]; bl = bl + T * f.bg[2]; }
    store_pixel(out, out_index(f.out_tiles, wt, x, y, f.H, f.tile_w, f.tile_h), f.out_rgb, r, g, bl);
    if (STATS == 2) count_work(stats, st_g, st_b, st_it);
}

// ------------------------------------------------------------------------------------------------
// TEST march along a volume axis (the reference's default camera looks along z; every view whose
// inverse-view matrix leaves the two other coordinates of p fixed along the ray -- host-checked with
// the other conditions, make_test).  For march axis a and fixed axes b < c: iv[8+b] = iv[8+c] = 0
// make iv[8+r] q1z + iv[12+r] = iv[12+r] for every sample bit for bit (a zero product is a signed
// zero, and iv[12+r] is not -0), so p_b and p_c -- and with them the corner lines (int)p_b,
// (int)(p_b + 1), ..., and the weights -- are constant along the ray, exactly; only p_a moves.
//
// getColorFromNF (kernel.cu:124-175) lerps the 8 classified corners in y, then x, then z.  Along z
// (AX = 2) z1 = lerp(lerp(c(x0,y0,i0z), c(x0,y1,i0z), dy), lerp(c(x1,y0,i0z), c(x1,y1,i0z), dy), dx)
// is a function of the plane index i0z alone (dx, dy fixed), and z2 the same at i1z = (int)(p_z + 1).
// So a ray carries its current plane pair (planes ja and ja + 1) from sample to sample: when p_a
// enters the next voxel the upper plane becomes the lower one and ONE new plane is computed; and a
// plane is a pure function of its 4 corner classes (the bytes of the 4 corner lines at index j, with
// the reference's flat-index wrap: line base + j * stride), so a plane whose class tuple equals its
// neighbour's is that neighbour's value -- no TF reads, no lerps.  The same operations on the same
// values as the reference's full evaluation, so frames are unchanged bit for bit (exact mode) --
// memoisation, not approximation.  What a plane holds in exact mode follows the reference's order:
//   z (AX 2): the y-then-x lerp of the plane (1 value); per sample the z lerp;
//   x (AX 0): the y lerps at z0 and z1 (2 values); per sample the two x lerps and the z lerp;
//   y (AX 1): the 4 classified colours (x0|x1, z0|z1); per sample the 4 y lerps, 2 x lerps, z lerp.
// Front to back (ERT, within its tolerance) a plane is the bilinear form of its 4 colours with the
// per-ray weights of the fixed axes, fused, and a sample one lerp along a -- for every axis.
// Class bytes: along z one 8-byte window per corner row (4 unaligned dwordx2 loads per 8 planes);
// along x or y the two z corners of a line pair are one unaligned dword (2 loads per plane).  Bytes
// past the volume are the zero pad / out-of-range zeros = class 0 = TF(0), the reference's
// idx < total guard.  A sample whose corners are all class 0 (TF(0), alpha 0) is an exact no-op.
// p_a itself is the same for every ray of the frame (host: iv[a] = iv[4+a] = 0 make A_a a signed
// zero, and A_a + u = u for u != 0, while u = +-0 gives tv_aa (+-0) + tv[12+a] = tv[12+a] != 0), so
// each workgroup tabulates (int)p_a, (int)(p_a + 1) and the weight p_a - (int)p_a per sample once,
// with the reference's expressions, and the march reads one LDS entry per sample.
// ESS: the ray's 4 corner lines' masks of occupied cells along a (test_columns_kernel) -- every
// other sample has class-0 corners -- with exact jumps to the next occupied cell (alpha-0 samples
// are exact no-ops of either blend, so every mode skips them).
// ------------------------------------------------------------------------------------------------
template <bool F2B, int AX>
struct AxisPlane {   // what a memoised plane holds (see above)
    static constexpr int NV = F2B || AX == 2 ? 1 : (AX == 0 ? 2 : 4);
    float4 v[NV];
};

#ifndef VR_TEST_AXIS_LOCK
#define VR_TEST_AXIS_LOCK 1
#endif
// waves per SIMD of the axis march: back to front (exact, ESS alone) capped at 7 (72 VGPRs, 12 B of
// spills): exact 0.183 -> 0.178-0.180 ms, ESS 0.186 -> 0.180-0.183 ms; front to back left to the
// compiler's 6 (74 VGPRs; 7 measured within noise) -- round 6, profiles/r6_ab/ab22_*.log
#ifndef VR_AXIS_WAVES
#define VR_AXIS_WAVES 1
#endif
#ifndef VR_AXIS_WAVES_B2F
#define VR_AXIS_WAVES_B2F 7
#endif
template <bool F2B, bool ESS, bool UP, int AX, int STATS = 0, bool LOCK = VR_TEST_AXIS_LOCK != 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(F2B ? VR_AXIS_WAVES : VR_AXIS_WAVES_B2F))) void test_axis_kernel(TestFrame f, const WorkTile* __restrict__ work,
                                                        const uint8_t* __restrict__ cls,
                                                        const float4* __restrict__ tf_rgba, int n_tf,
                                                        const unsigned long long* __restrict__ tcol,
                                                        float4* __restrict__ out,
                                                        unsigned long long* __restrict__ stats,
                                                        const int32_t* __restrict__ ztab_g, int ztab_words) {
#ifndef VR_AXIS_K
#define VR_AXIS_K 8
#endif
    static_assert(VR_AXIS_K <= 16, "the host table's slack covers 16 entries past the last");
    // samples between ERT / empty-cell checks (4: 3-5 % slower, round 4; 16: 3-5 % slower, round 5;
    // lockstep, round 6: 4 +4 %, 16 +13 % on C3 TEST default ESS + ERT, profiles/r6_ab/ab15_*.log)
    constexpr int K = VR_AXIS_K;
    constexpr int B = AX == 0 ? 1 : 0, C = AX == 2 ? 1 : 2;   // the fixed axes, b < c
    using PV = AxisPlane<F2B, AX>;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float4* s_tf = reinterpret_cast<float4*>(smem);
    // per-sample table of the march axis: x = (int)p_a | ((int)(p_a + 1) - (int)p_a) << 29, or -1
    // outside [0, d_a) (the host requires d_a < 2^28, so i0 never reaches the delta bits);
    // y = the bits of p_a - (int)p_a
    int2* s_ztab = reinterpret_cast<int2*>(smem + (size_t)n_tf * sizeof(float4));
    // ESS: per sample the cell of (int)p_a (-1 below the volume, tnca at or past its top: monotone
    // in s, p_a being a monotone function of s), and per cell the first sample in march order whose
    // cell is that cell or beyond it in the direction of travel (F2B: S if none; B2F: -1 if none) --
    // a jump to the next occupied cell of the ray's lines is one LDS read
    int8_t* s_zcel = reinterpret_cast<int8_t*>(s_ztab + f.S);
    int32_t* s_zent = reinterpret_cast<int32_t*>(s_zcel + ((size_t)f.S + 3) / 4 * 4);
    const int tca = f.tca[AX], tnca = f.tnca[AX];
    const float fda = AX == 0 ? f.fd1 : (AX == 1 ? f.fd2 : f.fd3);
    // the TF entry and the work tile in one round of loads; a culled work tile (or a background-only
    // workgroup) stores the background and leaves before the tables are built
    // (unconditional, index clamped; stored only for threadIdx.x < n_tf <= kMaxTf = kWgThreads, host)
    const float4 tfv = tf_rgba[(int)threadIdx.x < n_tf ? (int)threadIdx.x : 0];
    // the frame constants the exits branch on, loaded in the first round (vrc_march_kernel)
    asm volatile("" ::"s"(f.out_tiles), "s"(f.bg_first), "s"(f.n_work), "s"(f.n_hull), "s"(f.W), "s"(f.H));
    // the host's copy of the frame's tables (ztab_g: the LDS image from s_ztab on, ztab_words int32
    // words, make_test_axis_table in vr_api.cpp -- the same expressions as the build below), staged
    // 16 B per thread per load in the first round (buffer and LDS carry 16 B of slack); without it
    // every workgroup builds the tables (~6 integer divisions and ~40 float ops per thread)
    const int zt4 = (ztab_words + 3) >> 2;
    int4 zq[2];
#ifndef VR_AXIS_SLOAD
#define VR_AXIS_SLOAD 1
#endif
    // (lockstep front to back with the host's copy: the march reads it by scalar loads, no LDS copy)
    constexpr bool ZSK = VR_AXIS_SLOAD && F2B && LOCK;
    if (ztab_g && !ZSK) {
        const __amdgpu_buffer_rsrc_t zrs = uniform_rsrc(ztab_g, zt4 * 16);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const auto w = __builtin_amdgcn_raw_buffer_load_b128(zrs, ((int)threadIdx.x + u * kWgThreads) * 16, 0, 0);
            zq[u] = make_int4((int)w[0], (int)w[1], (int)w[2], (int)w[3]);
        }
    }
    const int b = (int)blockIdx.x;
    const WorkTile wt = work[b < f.n_work ? b : 0];   // (unconditional, see test_march_kernel)
    if (b >= f.n_work) return;
    if (test_background(f, work, wt, out)) return;
    if ((int)threadIdx.x < n_tf) s_tf[threadIdx.x] = tfv;
    if (ztab_g && !ZSK) {
        int4* zd = reinterpret_cast<int4*>(s_ztab);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int i = (int)threadIdx.x + u * kWgThreads;
            if (i < zt4) zd[i] = zq[u];
        }
        for (int i = (int)threadIdx.x + 2 * kWgThreads; i < zt4; i += kWgThreads)
            zd[i] = reinterpret_cast<const int4*>(ztab_g)[i];
    }
    auto pa_at = [&](int s) -> float {
        const float q1z = f.mc[10] * (float)s + f.mc[14];
        const float q2 = 0.0f + (f.iv[8 + AX] * q1z + f.iv[12 + AX] * 1.0f);   // A_a = +-0 (see above)
        return f.tv[5 * AX] * q2 + f.tv[12 + AX];
    };
    auto cell_of = [&](float pa) -> int {
        const bool in = pa >= 0.0f && pa < fda;
        return in ? (int)pa / tca : (pa < 0.0f ? -1 : tnca);
    };
    for (int s = threadIdx.x; !ztab_g && s < f.S; s += kWgThreads) {
        const float pa = pa_at(s);
        const int i0 = (int)pa, i1 = (int)(pa + 1.0f);
        const bool in = pa >= 0.0f && pa < fda;
        s_ztab[s] = make_int2(in ? (i0 | ((i1 - i0) << 29)) : -1, __float_as_int(pa - (float)(int)pa));
        if (ESS) s_zcel[s] = (int8_t)cell_of(pa);
    }
    // cells grow in march order when p_a does (F2B: UP; B2F: UP means p_a falls with s)
    constexpr bool cells_up = UP;
    if (ESS && !ztab_g) {
        // s_zent[c] = the first sample in march order whose cell is c or beyond it in the direction
        // of travel (F2B: S if none; B2F: -1 if none).  The cell h(m) of the m-th sample in march
        // order is monotone (p_a is), non-decreasing after a sign flip when cells fall (h' = +-h), so
        // entry c is the sample m where h'(m - 1) < c' <= h'(m) (c' = +-c): each sample writes the
        // cells its step crosses, threads over cells write those at or before the first sample's
        // cell and past the last one's -- every entry written once, in the same pass as the table
        // (round 4: a binary search per cell after one more barrier; the same entries)
        auto hp = [&](int s) { const int h = cell_of(pa_at(s)); return cells_up ? h : -h; };
        const int s_first = F2B ? 0 : f.S - 1, s_last = F2B ? f.S - 1 : 0, none = F2B ? f.S : -1;
        const int h_first = hp(s_first), h_last = hp(s_last);
        for (int c = threadIdx.x; c < tnca; c += kWgThreads) {
            const int cp = cells_up ? c : -c;
            if (cp <= h_first) s_zent[c] = s_first;
            else if (cp > h_last) s_zent[c] = none;
        }
        for (int s = threadIdx.x; s < f.S; s += kWgThreads) {
            if (s == s_first) continue;
            const int h0 = hp(F2B ? s - 1 : s + 1), h1 = hp(s);   // the previous sample in march order, this one
            for (int cp = h0 + 1; cp <= h1; ++cp) {
                const int c = cells_up ? cp : -cp;
                if (c >= 0 && c < tnca) s_zent[c] = s;
            }
        }
    }
    __syncthreads();
    int x, y;
    ray_of_thread(wt, x, y);
    const bool lane_ok = x < f.W && y < f.H;
    if (!LOCK && !lane_ok) return;   // (LOCK: after the wave's column mask, below)

    // SEP position of test_march_kernel: q1 = (mc0 x + mc12, mc5 y + mc13, mc10 s + mc14),
    // q2_r = A_r + (iv_{8+r} q1z + iv_{12+r}), p_r = tv_rr q2_r + tv_{12+r}
    const float fx = (float)x, fy = (float)y;
    const float q1x = f.mc[0] * fx + f.mc[12], q1y = f.mc[5] * fy + f.mc[13];
    float A[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) A[r] = f.iv[r] * q1x + f.iv[4 + r] * q1y;
    const float q1z0 = f.mc[10] * 0.0f + f.mc[14];
    const float pb = f.tv[5 * B] * (A[B] + (f.iv[8 + B] * q1z0 + f.iv[12 + B] * 1.0f)) + f.tv[12 + B];
    const float pc = f.tv[5 * C] * (A[C] + (f.iv[8 + C] * q1z0 + f.iv[12 + C] * 1.0f)) + f.tv[12 + C];
    const float fd[3] = {f.fd1, f.fd2, f.fd3};

    float r, g, bl, T = 1.0f;
    if (F2B) { r = 0.0f; g = 0.0f; bl = 0.0f; }
    else { r = f.bg[0]; g = f.bg[1]; bl = f.bg[2]; }
    // a ray whose (p_b, p_c) is outside the volume samples only TF(0) (transparent: host-checked)
    const bool in_bc = pb >= 0.0f && pb < fd[B] && pc >= 0.0f && pc < fd[C];
    // its clip range: p_a(s) is the same for every ray, so the host clipped the march axis once per
    // frame (make_test: ax_sb / ax_se, the per-ray double-precision clip of round 4 -- ~50 FP64
    // operations per wave -- bit for bit); the fixed axes' part of that clip is in_bc itself
    const int s_begin = in_bc ? f.ax_sb : 0;
    int s_end = in_bc ? f.ax_se : 0;
    // the 4 corner lines (b0|b1, c0|c1) as flat indices of p_a = 0 (host: total + d2 d3 + d3 + 1 < 2^31)
    const int i0b = (int)pb, i1b = (int)(pb + 1.0f), i0c = (int)pc, i1c = (int)(pc + 1.0f);
    const float wb = pb - (float)(int)pb, wc = pc - (float)(int)pc;
    const int d3 = (int)f.d3, d23 = (int)(f.d2 * f.d3);
    const int sB = B == 0 ? d23 : d3, sC = C == 1 ? d3 : 1;   // flat-index strides of the fixed axes
    const int sA = AX == 0 ? d23 : (AX == 1 ? d3 : 1);        // ... and of the march axis
    const int rb0 = i0b * sB + i0c * sC, rb1 = i0b * sB + i1c * sC;
    const int rb2 = i1b * sB + i0c * sC, rb3 = i1b * sB + i1c * sC;
    // ESS: the occupied cells of the ray's 4 corner lines, one mask per ray
    unsigned long long colmask = 0;
    if (ESS && in_bc && lane_ok) {
        const unsigned long long* tc = tcol + f.tcol_base[AX];
        const int pitch = f.tcol_pitch[AX];
        colmask = tc[(size_t)i0b * pitch + i0c] | tc[(size_t)i0b * pitch + i1c] | tc[(size_t)i1b * pitch + i0c] |
                  tc[(size_t)i1b * pitch + i1c];
        if (colmask == 0ull) s_end = s_begin;   // every sample of the ray has class-0 corners
    }
    // LOCK: the wave marches one sample sequence (p_a(s), hence the plane index, is the same for every
    // ray of the frame): the union of its rays' occupied cells, every plane transition a wave-uniform
    // branch (see the loop below)
    unsigned long long wmask = colmask;
    if (LOCK && ESS) {
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) wmask |= __shfl_xor(wmask, o);
        // (every lane holds the union now; read back through readfirstlane so the compiler sees a
        // wave-uniform value -- from the shuffles it is a VGPR, which made every test on it, and with
        // them the plane index and window base the march carries, exec-masked branches)
#ifndef VR_AXIS_UNIMASK
#define VR_AXIS_UNIMASK 1
#endif
        if (VR_AXIS_UNIMASK)
            wmask = ((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(wmask >> 32)) << 32) |
                    (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)wmask);
    }
    if (LOCK && !lane_ok) return;
    const __amdgpu_buffer_rsrc_t trs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(cls), (short)0, (int)f.total + kClsPad / 4, 0x00020000);

    unsigned st_g = 0, st_b = 0, st_it = 0;   // STATS: gathers, bytes, samples evaluated
    // along z: class window, bytes [jw, jw + 8) of each corner row
    uint64_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;
    int jw = INT32_MIN / 2;
    auto ensure = [&](int lo, int hi) {   // hi - lo <= 2
        if (AX == 2 && (lo < jw || hi > jw + 7)) {
            if (STATS) { st_g += 4; st_b += 32; }
            jw = UP ? lo : max(hi - 7, 0);
            const auto v0 = __builtin_amdgcn_raw_buffer_load_b64(trs, rb0 + jw, 0, 0);
            const auto v1 = __builtin_amdgcn_raw_buffer_load_b64(trs, rb1 + jw, 0, 0);
            const auto v2 = __builtin_amdgcn_raw_buffer_load_b64(trs, rb2 + jw, 0, 0);
            const auto v3 = __builtin_amdgcn_raw_buffer_load_b64(trs, rb3 + jw, 0, 0);
            w0 = ((uint64_t)v0[1] << 32) | v0[0];
            w1 = ((uint64_t)v1[1] << 32) | v1[0];
            w2 = ((uint64_t)v2[1] << 32) | v2[0];
            w3 = ((uint64_t)v3[1] << 32) | v3[0];
        }
    };
    const unsigned dzc = (unsigned)(i1c - i0c) * 8u;   // along x / y: bit offset of the c1 corner (1 or 2 bytes)
    auto key_at = [&](int j) -> uint32_t {   // the 4 corner classes of plane j: (b0c0, b0c1, b1c0, b1c1)
#ifndef VR_AXIS_PERM
#define VR_AXIS_PERM 0
#endif
        if (AX == 2 && VR_AXIS_PERM) {
            // byte k = j - jw of the four windows by two byte permutes (v_perm_b32: selector bytes 0-3
            // pick the second operand's bytes, 4-7 the first's, 0x0c gives 0) from the half holding it.
            // Off: 7 VALU instead of ~11 per key and 70 VGPRs instead of 74, yet C3 TEST default ESS + ERT
            // 0.105 -> 0.111 ms (round 6, profiles/r6_ab/ab12_*.log)
            const int k = j - jw;
            const bool hi = k >= 4;
            const uint32_t kb = (uint32_t)(k & 3);
            const uint32_t a0 = hi ? (uint32_t)(w0 >> 32) : (uint32_t)w0, a1 = hi ? (uint32_t)(w1 >> 32) : (uint32_t)w1;
            const uint32_t a2 = hi ? (uint32_t)(w2 >> 32) : (uint32_t)w2, a3 = hi ? (uint32_t)(w3 >> 32) : (uint32_t)w3;
            return __builtin_amdgcn_perm(a1, a0, 0x0c0c0000u | ((4u + kb) << 8) | kb) |
                   __builtin_amdgcn_perm(a3, a2, ((4u + kb) << 24) | (kb << 16) | 0x0c0cu);
        }
        if (AX == 2) {
            const unsigned sh = (unsigned)(j - jw) * 8u;
            return (uint32_t)((w0 >> sh) & 0xffu) | ((uint32_t)((w1 >> sh) & 0xffu) << 8) |
                   ((uint32_t)((w2 >> sh) & 0xffu) << 16) | ((uint32_t)((w3 >> sh) & 0xffu) << 24);
        }
        // (c is z here: the c0 and c1 corners of a line pair are one unaligned dword)
        if (STATS) { st_g += 2; st_b += 8; }
        const uint32_t u0 = __builtin_amdgcn_raw_buffer_load_b32(trs, rb0 + j * sA, 0, 0);
        const uint32_t u1 = __builtin_amdgcn_raw_buffer_load_b32(trs, rb2 + j * sA, 0, 0);
        return (u0 & 0xffu) | (((u0 >> dzc) & 0xffu) << 8) | ((u1 & 0xffu) << 16) | (((u1 >> dzc) & 0xffu) << 24);
    };
    // front to back (ERT, within its tolerance): the plane's bilinear form with the per-ray weights
    // (1-wb)(1-wc), (1-wb)wc, wb(1-wc), wb wc, fused -- a reassociation of the lerps
    const float b00 = (1.0f - wb) * (1.0f - wc), b01 = (1.0f - wb) * wc, b10 = wb * (1.0f - wc), b11 = wb * wc;
    auto plane = [&](uint32_t key) -> PV {   // kernel.cu:162-173 for one plane
        const float4 c00 = s_tf[key & 0xffu], c01 = s_tf[(key >> 8) & 0xffu];
        const float4 c10 = s_tf[(key >> 16) & 0xffu], c11 = s_tf[key >> 24];
        PV P;
        if (F2B) {   // the fused bilinear form, two channels per packed op
            const f2 B00 = {b00, b00}, B01 = {b01, b01}, B10 = {b10, b10}, B11 = {b11, b11};
            const f2 lo = __builtin_elementwise_fma(
                f2{c11.x, c11.y}, B11,
                __builtin_elementwise_fma(f2{c10.x, c10.y}, B10,
                                          __builtin_elementwise_fma(f2{c01.x, c01.y}, B01, f2{c00.x, c00.y} * B00)));
            const f2 hi = __builtin_elementwise_fma(
                f2{c11.z, c11.w}, B11,
                __builtin_elementwise_fma(f2{c10.z, c10.w}, B10,
                                          __builtin_elementwise_fma(f2{c01.z, c01.w}, B01, f2{c00.z, c00.w} * B00)));
            P.v[0] = make_float4(lo.x, lo.y, hi.x, hi.y);
        } else if (AX == 2) {   // y (= c) lerps, then x (= b)
            P.v[0] = lerp4<false>(lerp4<false>(c00, c01, wc), lerp4<false>(c10, c11, wc), wb);
        } else if (AX == 0) {   // the y (= b) lerps at z0 and z1
            P.v[0] = lerp4<false>(c00, c10, wb);
            P.v[PV::NV > 1 ? 1 : 0] = lerp4<false>(c01, c11, wb);
        } else {                // y moves: the classified colours themselves
            P.v[0] = c00;
            P.v[PV::NV > 1 ? 1 : 0] = c01;
            P.v[PV::NV > 2 ? 2 : 0] = c10;
            P.v[PV::NV > 3 ? 3 : 0] = c11;
        }
        return P;
    };
    // a sample from its lower plane P and upper plane Q with the march-axis weight w
    auto sample = [&](const PV& P, const PV& Q, float w) -> float4 {
        if (F2B || AX == 2) return lerp4<F2B>(P.v[0], Q.v[0], w);
        if (AX == 0) {   // x lerps at z0 and z1, then z (= c)
            const float4 z1 = lerp4<false>(P.v[0], Q.v[0], w);
            const float4 z2 = lerp4<false>(P.v[PV::NV > 1 ? 1 : 0], Q.v[PV::NV > 1 ? 1 : 0], w);
            return lerp4<false>(z1, z2, wc);
        }
        // y moves: y lerps of the 4 (x, z) lines, x (= b) lerps, then z (= c)
        const float4 y1 = lerp4<false>(P.v[0], Q.v[0], w);
        const float4 y2 = lerp4<false>(P.v[PV::NV > 1 ? 1 : 0], Q.v[PV::NV > 1 ? 1 : 0], w);
        const float4 y3 = lerp4<false>(P.v[PV::NV > 2 ? 2 : 0], Q.v[PV::NV > 2 ? 2 : 0], w);
        const float4 y4 = lerp4<false>(P.v[PV::NV > 3 ? 3 : 0], Q.v[PV::NV > 3 ? 3 : 0], w);
        const float4 z1 = lerp4<false>(y1, y3, wb), z2 = lerp4<false>(y2, y4, wb);
        return lerp4<false>(z1, z2, wc);
    };

    int ja = INT32_MIN / 2;   // planes ja and ja + 1: classes k0, k1, values P0, P1
    uint32_t k0 = 0, k1 = 0;
    PV P0, P1;
#pragma unroll
    for (int i = 0; i < PV::NV; ++i) P0.v[i] = P1.v[i] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    // front to back: a sample is P0 + wa (P1 - P0), the difference kept with the planes (one fma per
    // channel per sample; the lerp reassociated within the ERT tolerance, like the fused plane)
    float4 D01 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    auto sub4 = [](float4 a, float4 b) { return make_float4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w); };
    if constexpr (LOCK) {
        // Lockstep: every active lane of the wave (in_bc, and ESS: an occupied cell on its corner lines)
        // shares the host's clip range [ax_sb, ax_se) and marches the same samples; the table entries,
        // the plane index and the window base are wave-uniform (scalar registers), so the plane
        // transitions are scalar branches instead of exec-mask juggling per lane.  The empty-cell jumps
        // follow the union of the lanes' masks: a lane in one of its own empty cells composites
        // class-0 samples, TF(0) with alpha 0 -- exact no-ops of either blend -- so exact frames are
        // bit for bit those of the per-lane march; front to back checks ERT at other batch ends
        // (within its tolerance).  Inactive and finished lanes never composite.
#ifndef VR_AXIS_NOMEMO
#define VR_AXIS_NOMEMO 0
#endif
        // (NOMEMO: every lane computes the new plane, no per-lane test of its class tuple)
        constexpr bool NOMEMO = VR_AXIS_NOMEMO != 0;
        const bool act = in_bc && (!ESS || colmask != 0ull);
        bool dl = !act;   // this lane takes no more samples
        const int sb = f.ax_sb, se = f.ax_se;
        int su = F2B ? sb : se - 1;
        const bool any_act = __any(act);
        bool wdone = !any_act || (F2B ? (su >= se) : (su < sb));
        // The batch's K table entries read together at its start: front to back by scalar loads from
        // the host's copy (ztab_g, K int2 = one s_load_dwordx16; the buffer carries 128 B of slack past
        // the last entry, make_test_axis_table), otherwise K LDS reads issued before the first is used
        // -- read one per sample, each waited for in turn (an LDS round trip per sample, in series)
        typedef const __attribute__((address_space(4))) int32_t cint;
        const bool zs = VR_AXIS_SLOAD && F2B && ztab_g != nullptr;
        cint* zg = (cint*)ztab_g;
        const int S_ = f.S;
        while (!wdone) {
            int exk[K], eyk[K];
            if (VR_AXIS_SLOAD && zs) {
                // (issued with the cell word below: one scalar round trip per batch; a jump discards them)
                cint* zp = zg + 2 * su;
#pragma unroll
                for (int k = 0; k < K; ++k) { exk[k] = zp[2 * k]; eyk[k] = zp[2 * k + 1]; }
            }
            if (ESS) {
                int cm;
                if (VR_AXIS_SLOAD && zs) {   // (the cell bytes follow the 2 S words of entries)
                    const int w = zg[2 * S_ + (su >> 2)];
                    cm = (int)(int8_t)(uint32_t)((uint32_t)w >> (8 * (su & 3)));
                } else {
                    cm = __builtin_amdgcn_readfirstlane((int)s_zcel[su]);
                }
                const bool occupied = (unsigned)cm < (unsigned)tnca && ((wmask >> cm) & 1ull);
                if (!occupied) {
                    const unsigned long long rest =
                        cells_up ? (cm >= 63 ? 0ull : wmask >> (cm + 1))
                                 : (cm <= 0 ? 0ull : (cm >= 64 ? wmask : wmask & ((1ull << cm) - 1ull)));
                    if (rest == 0ull) break;
                    const int nxt = cells_up ? cm + 1 + __builtin_ctzll(rest) : 63 - __builtin_clzll(rest);
                    // (the entry words follow the cell bytes, padded to 4 B)
                    su = (VR_AXIS_SLOAD && zs) ? zg[2 * S_ + ((S_ + 3) >> 2) + nxt]
                                               : __builtin_amdgcn_readfirstlane(s_zent[nxt]);
                    wdone = F2B ? (su >= se) : (su < sb);
                    continue;
                }
            }
            if (STATS) st_it += act ? K : 0;
            if (VR_AXIS_SLOAD && !zs) {
                int2 ek[K];
#pragma unroll
                for (int k = 0; k < K; ++k) {   // (index clamped into the table: entries past the clip are unused)
                    const int sk = F2B ? su + k : su - k;
                    ek[k] = s_ztab[min(max(sk, 0), S_ - 1)];
                }
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    exk[k] = __builtin_amdgcn_readfirstlane(ek[k].x);
                    eyk[k] = __builtin_amdgcn_readfirstlane(ek[k].y);
                }
            }
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int sk = F2B ? su + k : su - k;
                if (F2B ? (sk >= se) : (sk < sb)) break;
                const int ex = VR_AXIS_SLOAD ? exk[k] : __builtin_amdgcn_readfirstlane(s_ztab[sk].x);
                const int ey = VR_AXIS_SLOAD ? eyk[k] : __builtin_amdgcn_readfirstlane(s_ztab[sk].y);
                if (ex < 0) continue;   // outside the volume: TF(0), alpha 0
                const int i0a = ex & 0x1fffffff, i1a = i0a + (ex >> 29);
                const float wa = __int_as_float(ey);
                if (i0a != ja) {
                    if (UP && i0a == ja + 1) {
                        ensure(ja + 1, ja + 2);
                        ja = i0a; P0 = P1; k0 = k1;
                        k1 = key_at(ja + 1);
                        if (NOMEMO || k1 != k0) P1 = plane(k1);
                    } else if (!UP && i0a == ja - 1) {
                        ensure(ja - 1, ja);
                        ja = i0a; P1 = P0; k1 = k0;
                        k0 = key_at(ja);
                        if (NOMEMO || k0 != k1) P0 = plane(k0);
                    } else {
                        ja = i0a;
                        ensure(ja, ja + 1);
                        k0 = key_at(ja);
                        k1 = key_at(ja + 1);
                        P0 = plane(k0);
                        P1 = (!NOMEMO && k1 == k0) ? P0 : plane(k1);
                    }
                    if (F2B) D01 = sub4(P1.v[0], P0.v[0]);
                }
                uint32_t k2 = k1;
                PV z2 = P1;
                float4 d = D01;
                if (i1a != ja + 1) {
                    ensure(ja, i1a);
                    k2 = key_at(i1a);
                    if (NOMEMO || k2 != k1) z2 = plane(k2);
                    if (F2B) d = sub4(z2.v[0], P0.v[0]);
                }
                if (!dl) {
                    const float4 cf = F2B ? make_float4(fmaf(wa, d.x, P0.v[0].x), fmaf(wa, d.y, P0.v[0].y),
                                                        fmaf(wa, d.z, P0.v[0].z), fmaf(wa, d.w, P0.v[0].w))
                                          : sample(P0, z2, wa);
                    const float a = cf.w;
                    if (F2B) {
                        const float wt_ = T * a;
                        r = fmaf(wt_, cf.x, r); g = fmaf(wt_, cf.y, g); bl = fmaf(wt_, cf.z, bl);
                        T = T * (1.0f - a);
                    } else {
                        r = r * (1 - a) + cf.x * a;
                        g = g * (1 - a) + cf.y * a;
                        bl = bl * (1 - a) + cf.z * a;
                    }
                }
            }
            if (F2B) {
                dl = dl || T < f.ert_eps;
                if (__all(dl)) break;
            }
            su = F2B ? su + K : su - K;
            wdone = F2B ? (su >= se) : (su < sb);
        }
    } else {
    int s = F2B ? s_begin : s_end - 1;
    bool done = F2B ? (s >= s_end) : (s < s_begin);
    while (!done) {
        if (ESS) {   // an empty cell of the ray's corner lines: jump to the next occupied one
            const int cm = s_zcel[s];   // (s is inside the clip range here)
            const bool occupied = (unsigned)cm < (unsigned)tnca && ((colmask >> cm) & 1ull);
            if (!occupied) {
                // cells -1 / tnca (outside the volume) are empty; none left in the direction of
                // travel: every later sample has class-0 corners -- the ray is finished
                const unsigned long long rest =
                    cells_up ? (cm >= 63 ? 0ull : colmask >> (cm + 1))
                             : (cm <= 0 ? 0ull : (cm >= 64 ? colmask : colmask & ((1ull << cm) - 1ull)));
                if (rest == 0ull) break;
                const int nxt = cells_up ? cm + 1 + __builtin_ctzll(rest) : 63 - __builtin_clzll(rest);
                s = s_zent[nxt];
                done = F2B ? (s >= s_end) : (s < s_begin);
                continue;
            }
        }
        if (STATS) st_it += K;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int sk = F2B ? s + k : s - k;
            const bool valid = F2B ? (sk < s_end) : (sk >= s_begin);
            const int2 e = s_ztab[valid ? sk : s];
            // outside the clip or the volume: TF(0), alpha 0 -- an exact no-op in either blend
            if (!valid || e.x < 0) continue;
            const int i0a = e.x & 0x1fffffff, i1a = i0a + (e.x >> 29);
            const float wa = __int_as_float(e.y);
            if (i0a != ja) {
                if (UP && i0a == ja + 1) {            // next voxel up: the upper plane moves down
                    ensure(ja + 1, ja + 2);
                    ja = i0a; P0 = P1; k0 = k1;
                    k1 = key_at(ja + 1);
                    if (k1 != k0) P1 = plane(k1);
                } else if (!UP && i0a == ja - 1) {    // next voxel down: the lower plane moves up
                    ensure(ja - 1, ja);
                    ja = i0a; P1 = P0; k1 = k0;
                    k0 = key_at(ja);
                    if (k0 != k1) P0 = plane(k0);
                } else {                              // first sample, or after an empty-cell jump
                    ja = i0a;
                    ensure(ja, ja + 1);
                    k0 = key_at(ja);
                    k1 = key_at(ja + 1);
                    P0 = plane(k0);
                    P1 = k1 == k0 ? P0 : plane(k1);
                }
                if (F2B) D01 = sub4(P1.v[0], P0.v[0]);
            }
            // the upper corners: (int)(p_a + 1) is ja + 1, or ja + 2 when p_a + 1 rounds up to it
            uint32_t k2 = k1;
            PV z2 = P1;
            float4 d = D01;
            if (i1a != ja + 1) {
                ensure(ja, i1a);
                k2 = key_at(i1a);
                if (k2 != k1) z2 = plane(k2);
                if (F2B) d = sub4(z2.v[0], P0.v[0]);
            }
            // (a sample whose corners are all class 0 -- TF(0), alpha 0 -- composites as an exact
            // no-op: front to back r + (T 0) c = r, T (1 - 0) = T; back to front r (1 - 0) + c 0 = r.
            // No branch around it: round 4's `continue` there cost exec-mask juggling on every
            // sample, 3 % of the default-view TEST frame)
            const float4 cf = F2B ? make_float4(fmaf(wa, d.x, P0.v[0].x), fmaf(wa, d.y, P0.v[0].y),
                                                fmaf(wa, d.z, P0.v[0].z), fmaf(wa, d.w, P0.v[0].w))
                                  : sample(P0, z2, wa);
            const float a = cf.w;
            if (F2B) {
                const float wt_ = T * a;
                r = fmaf(wt_, cf.x, r); g = fmaf(wt_, cf.y, g); bl = fmaf(wt_, cf.z, bl);
                T = T * (1.0f - a);
            } else {
                r = r * (1 - a) + cf.x * a;
                g = g * (1 - a) + cf.y * a;
                bl = bl * (1 - a) + cf.z * a;
            }
        }
        if (F2B && T < f.ert_eps) done = true;
        s = F2B ? s + K : s - K;
        if (F2B ? (s >= s_end) : (s < s_begin)) done = true;
    }
    }   // !LOCK
    if (F2B) { r = r + T * f.bg[0]; g = g + T * f.bg[1]; bl = bl + T * f.bg[2]; }
    store_pixel(out, out_index(f.out_tiles, wt, x, y, f.H, f.tile_w, f.tile_h), f.out_rgb, r, g, bl);
    if (STATS == 2) count_work(stats, st_g, st_b, st_it);
}

// Occupancy of TEST macro cells: cell (cx, cy, cz) covers voxels [c*B, c*B + B + 1] per axis (the
// corners a sample in the cell can reach); occupied iff one of them has alpha > 0, or the range
// reaches an upper face (corner indices wrap there).
__global__ __launch_bounds__(256) void test_occupancy_kernel(const uint8_t* __restrict__ cls, int64_t d1, int64_t d2,
                                                             int64_t d3, int tcb, int nc1, int nc2, int nc3,
                                                             const uint8_t* __restrict__ alpha_nz,
                                                             unsigned long long* __restrict__ occ) {
    const int64_t ncells = (int64_t)nc1 * nc2 * nc3;
    const int64_t cell = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool occupied = false;
    if (cell < ncells) {
        const int c[3] = {(int)(cell / ((int64_t)nc2 * nc3)), (int)((cell / nc3) % nc2), (int)(cell % nc3)};
        const int64_t d[3] = {d1, d2, d3};
        int64_t lo[3], hi[3];
        for (int a = 0; a < 3; ++a) {
            lo[a] = (int64_t)c[a] << tcb;
            hi[a] = lo[a] + ((int64_t)1 << tcb) + 1;
            if (hi[a] >= d[a] - 1) occupied = true;
            hi[a] = hi[a] < d[a] - 1 ? hi[a] : d[a] - 1;
        }
        for (int64_t x = lo[0]; x <= hi[0] && !occupied; ++x)
            for (int64_t y = lo[1]; y <= hi[1] && !occupied; ++y) {
                const uint8_t* row = cls + (x * d2 + y) * d3;
                for (int64_t z = lo[2]; z <= hi[2]; ++z)
                    if (alpha_nz[row[z]]) { occupied = true; break; }
            }
    }
    const unsigned long long m = __ballot(occupied);
    if ((threadIdx.x & 63) == 0 && cell < ncells) occ[cell >> 6] = m;
}

// The TEST corner volume (TestFrame.cv): for every voxel idx, the classes of its 8 trilinear
// corners, corner kk = (x << 2 | y << 1 | z) at flat index idx + x d2 d3 + y d3 + z (kernel.cu:130-155:
// flat indices with only the idx < total guard -- class 0 past the end -- so a corner at a row's end
// wraps into the next row exactly as the reference reads it), CB bits each at bit CB corner_field(kk)
// (the z = 0 plane's four corners, then the z = 1 plane's): CB bytes
// per voxel, at byte CB idx (x-major, lay == nullptr) or at byte lay[x] + lay[d1 + y] +
// lay[d1 + d2 + z] (the 4 x 4 x 4 brick layout, vr_api.cpp classify).
template <int CB>
__global__ __launch_bounds__(256) void test_corner_kernel(const uint8_t* __restrict__ cls, int64_t total, int64_t d1,
                                                          int64_t d2, int64_t d3, const int32_t* __restrict__ lay,
                                                          uint8_t* __restrict__ out) {
    const int64_t d23 = d2 * d3;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t w = 0;
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) {
            const int64_t j = i + ((kk >> 2) & 1) * d23 + ((kk >> 1) & 1) * d3 + (kk & 1);
            w |= (uint64_t)(j < total ? cls[j] : 0) << (CB * corner_field(kk));
        }
        uint8_t* o = out + i * CB;   // (CB bits x 8 corners = CB bytes per voxel)
        if (lay) {
            const int64_t x = i / d23, y = (i / d3) % d2, z = i % d3;
            o = out + (lay[x] + lay[d1 + y] + lay[d1 + d2 + z]);
        }
        if (CB == 2) *reinterpret_cast<uint16_t*>(o) = (uint16_t)w;
        else if (CB == 4) *reinterpret_cast<uint32_t*>(o) = (uint32_t)w;
        else *reinterpret_cast<uint64_t*>(o) = w;
    }
}

// Column masks of the TEST class volume for axis views (TestFrame.tca): march axis a, one thread
// per corner line (u, v) of the two other axes (each in [0, d + 2)), bit c = some byte at flat index
// u s_u + v s_v + t s_a, t in [c tca, c tca + tca + 1], has alpha > 0.  Flat indices as the march
// reads them: an index past a row runs into the next one and anything at or past `total` is class 0
// (the reference's idx < total guard), so the mask covers exactly the bytes a sample of the cell
// can touch.
__global__ __launch_bounds__(256) void test_columns_kernel(const uint8_t* __restrict__ cls, int64_t total,
                                                           int64_t nu, int64_t nv, int64_t su, int64_t sv, int64_t sa,
                                                           int tca, int tnca, const uint8_t* __restrict__ alpha_nz,
                                                           unsigned long long* __restrict__ cols) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nu * nv) return;
    const int64_t base = (i / nv) * su + (i % nv) * sv;
    unsigned long long m = 0;
    for (int c = 0; c < tnca; ++c) {
        bool any = false;
        for (int64_t t = (int64_t)c * tca; t <= (int64_t)c * tca + tca + 1; ++t) {
            const int64_t idx = base + t * sa;
            any = any || (idx < total && alpha_nz[cls[idx]]);
        }
        if (any) m |= 1ull << c;
    }
    cols[i] = m;
}

// ------------------------------------------------------------------------------------------------
// Launch wrappers (called from vr_api.cpp)
// ------------------------------------------------------------------------------------------------
hipError_t launch_test_march(const TestFrame& f, const WorkTile* work, const int32_t* order, int n_blocks,
                             const uint8_t* cls, const float4* tf, int n_tf, const uint32_t* occ, float4* out,
                             hipStream_t st, const unsigned long long* tcol, const uint8_t* cvol, const int32_t* clay,
                             unsigned long long* count, const int32_t* ztab, int ztab_words) {
    const bool f2b = (f.flags & 2) != 0, ess = (f.flags & 1) != 0 && f.zero_transparent && occ != nullptr;
#ifndef VR_TEST_K
#define VR_TEST_K 4
#endif
    constexpr int K = VR_TEST_K;   // samples per TEST batch (general views)
    // the corner volume needs class 0 = TF(0), 32-bit indices (host: built only then) and 24-bit
    // index products (d1, d2 d3 < 2^24: the march's __umul24 offsets)
    const int cv = (cvol != nullptr && !f.idx64 && f.cls0 == 0 && f.sep && f.mul24) ? f.cv : 0;
    // (SEP: + the per-frame B table, 16 B per sample of [-K, S + K); a bricked corner volume: + its
    // offset tables, 4 B per voxel row of each axis)
    size_t lds = (((size_t)n_tf * sizeof(float4) + ((ess && f.occ_lds) ? (size_t)f.occ_words * 4 : 0) + 15) / 16 *
                  16) + ((f.sep && f.sep_tab) ? (size_t)(f.S + 2 * K) * sizeof(float4) : 0) +
                 ((cv != 0 && cv < 16) ? (size_t)(f.d1 + f.d2 + f.d3) * 4 : 0);
    // the plane table (front to back, 2-bit corner classes): + 16 KB, while the workgroup stays within
    // a fifth of the CU's 160 KB (the 5 workgroups per CU its registers allow; longer rays' B tables
    // keep the TF reads)
    const bool pt = f2b && (cv == 2 || cv == 18) && lds + kPtBytes <= 32768;
    if (pt) lds += kPtBytes;
    // axis plane march: the TF table, the axis table (8 B per sample), and with the column skip the
    // per-sample cells (1 B) and the cells' entry samples (4 B per cell)
    const bool ess_axz = f.zero_transparent && tcol != nullptr;
    const int ax = f.axt >= 0 ? f.axt : 2;
    const size_t lds_axz = (size_t)n_tf * sizeof(float4) + (size_t)f.S * 8 +
                           (ess_axz ? ((size_t)f.S + 3) / 4 * 4 + (size_t)f.tnca[ax] * 4 : 0) +
                           16;   // (a staged host table ends in a whole int4)
#define VR_TKP(F2B_, ESS_, I64_, SEP_, CV_, PT_)                                                                \
    do {                                                                                                        \
        if (count)                                                                                              \
            hipLaunchKernelGGL((test_march_kernel<F2B_, ESS_, I64_, K, SEP_, CV_, PT_, 2>), dim3(n_blocks),   \
                               dim3(kWgThreads), lds, st, f, work, order, cls, tf, n_tf, occ, out, cvol, clay, count); \
        else                                                                                                    \
            hipLaunchKernelGGL((test_march_kernel<F2B_, ESS_, I64_, K, SEP_, CV_, PT_, 0>), dim3(n_blocks),   \
                               dim3(kWgThreads), lds, st, f, work, order, cls, tf, n_tf, occ, out, cvol, clay, count); \
    } while (0)
#define VR_TK(F2B_, ESS_, I64_, SEP_, CV_) VR_TKP(F2B_, ESS_, I64_, SEP_, CV_, false)
    // (pt implies front to back: PT_ = F2B_ instantiates the table variant for F2B only)
#define VR_T(F2B_, ESS_)                                                                                        \
    if (f.idx64) { if (f.sep) VR_TK(F2B_, ESS_, true, true, 0); else VR_TK(F2B_, ESS_, true, false, 0); }     \
    else if (!f.sep) VR_TK(F2B_, ESS_, false, false, 0);                                                        \
    else if (cv == 18) { if (pt) VR_TKP(F2B_, ESS_, false, true, 18, F2B_); else VR_TK(F2B_, ESS_, false, true, 18); } \
    else if (cv == 20) VR_TK(F2B_, ESS_, false, true, 20);                                                      \
    else if (cv == 24) VR_TK(F2B_, ESS_, false, true, 24);                                                      \
    else if (cv == 2) { if (pt) VR_TKP(F2B_, ESS_, false, true, 2, F2B_); else VR_TK(F2B_, ESS_, false, true, 2); } \
    else if (cv == 4) VR_TK(F2B_, ESS_, false, true, 4);                                                        \
    else if (cv == 8) VR_TK(F2B_, ESS_, false, true, 8);                                                        \
    else VR_TK(F2B_, ESS_, false, true, 0)
#define VR_ZA(F2B_, ESS_, UP_, AX_)                                                                  \
    do {                                                                                             \
        if (count)                                                                                   \
            hipLaunchKernelGGL((test_axis_kernel<F2B_, ESS_, UP_, AX_, 2>), dim3(n_blocks), dim3(kWgThreads), lds_axz, st, \
                               f, work, cls, tf, n_tf, tcol, out, count, ztab, ztab_words);          \
        else                                                                                         \
            hipLaunchKernelGGL((test_axis_kernel<F2B_, ESS_, UP_, AX_, 0>), dim3(n_blocks), dim3(kWgThreads), lds_axz, st, \
                               f, work, cls, tf, n_tf, tcol, out, count, ztab, ztab_words);          \
    } while (0)
#define VR_Z(F2B_, ESS_, UP_)                                                                        \
    if (ax == 0) VR_ZA(F2B_, ESS_, UP_, 0); else if (ax == 1) VR_ZA(F2B_, ESS_, UP_, 1); else VR_ZA(F2B_, ESS_, UP_, 2)
    if (f.axt >= 0 && !order) {
        // the march direction along the axis in march order (F2B: s ascending).  Empty cells of the
        // ray's corner lines are skipped in every mode (alpha-0 samples are exact no-ops of either blend)
        const bool up = f2b ? f.axt_up != 0 : f.axt_up == 0;
        if (f2b) {
            if (ess_axz) { if (up) VR_Z(true, true, true); else VR_Z(true, true, false); }
            else { if (up) VR_Z(true, false, true); else VR_Z(true, false, false); }
        } else {
            if (ess_axz) { if (up) VR_Z(false, true, true); else VR_Z(false, true, false); }
            else { if (up) VR_Z(false, false, true); else VR_Z(false, false, false); }
        }
    } else if (f2b) {
        if (ess) { VR_T(true, true); } else { VR_T(true, false); }
    } else {
        if (ess) { VR_T(false, true); } else { VR_T(false, false); }
    }
#undef VR_Z
#undef VR_ZA
#undef VR_T
#undef VR_TK
#undef VR_TKP
    return hipGetLastError();
}

hipError_t launch_test_occupancy(const uint8_t* cls, int64_t d1, int64_t d2, int64_t d3, int tcb, int nc1, int nc2,
                                 int nc3, const uint8_t* alpha_nz, unsigned long long* occ, hipStream_t st) {
    const int64_t ncells = (int64_t)nc1 * nc2 * nc3;
    const int blocks = (int)((ncells + 255) / 256);
    hipLaunchKernelGGL(test_occupancy_kernel, dim3(blocks), dim3(256), 0, st, cls, d1, d2, d3, tcb, nc1, nc2, nc3,
                       alpha_nz, occ);
    return hipGetLastError();
}

// cb in {2, 4, 8} bits per class; lay == nullptr: x-major, else the brick tables
hipError_t launch_test_corners(const uint8_t* cls, int64_t total, int64_t d1, int64_t d2, int64_t d3, const int32_t* lay,
                               int cb, uint8_t* out, hipStream_t st) {
    const int blocks = (int)std::min<int64_t>((total + 255) / 256, 256 * 64);
    if (cb == 2) hipLaunchKernelGGL(test_corner_kernel<2>, dim3(blocks), dim3(256), 0, st, cls, total, d1, d2, d3, lay, out);
    else if (cb == 4) hipLaunchKernelGGL(test_corner_kernel<4>, dim3(blocks), dim3(256), 0, st, cls, total, d1, d2, d3, lay, out);
    else hipLaunchKernelGGL(test_corner_kernel<8>, dim3(blocks), dim3(256), 0, st, cls, total, d1, d2, d3, lay, out);
    return hipGetLastError();
}

// Faces of the class volume: flag = 1 when a voxel on one of the six faces (x, y or z at 0 or d - 1)
// is not class 0.  Every writer stores the same value (plain vector stores, no atomics).
__global__ __launch_bounds__(256) void test_faces_kernel(const uint8_t* __restrict__ cls, int64_t d1, int64_t d2,
                                                         int64_t d3, int32_t* __restrict__ flag) {
    const int64_t nx = d2 * d3, ny = d1 * d3, nz = d1 * d2;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nx + ny + nz;
         i += (int64_t)gridDim.x * blockDim.x) {
        int64_t a, b;   // the two flat indices of the voxel pair on opposite faces
        if (i < nx) {
            a = i;
            b = (d1 - 1) * nx + i;
        } else if (i < nx + ny) {
            const int64_t j = i - nx, x = j / d3, z = j % d3;
            a = x * nx + z;
            b = x * nx + (d2 - 1) * d3 + z;
        } else {
            const int64_t j = i - nx - ny, x = j / d2, y = j % d2;
            a = x * nx + y * d3;
            b = a + d3 - 1;
        }
        if ((cls[a] | cls[b]) != 0) flag[0] = 1;
    }
}

hipError_t launch_test_faces(const uint8_t* cls, int64_t d1, int64_t d2, int64_t d3, int32_t* flag, hipStream_t st) {
    const int64_t n = d2 * d3 + d1 * d3 + d1 * d2;
    const int blocks = (int)std::min<int64_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(test_faces_kernel, dim3(blocks), dim3(256), 0, st, cls, d1, d2, d3, flag);
    return hipGetLastError();
}

hipError_t launch_test_columns(const uint8_t* cls, int64_t total, int64_t nu, int64_t nv, int64_t su, int64_t sv,
                               int64_t sa, int tca, int tnca, const uint8_t* alpha_nz, unsigned long long* cols,
                               hipStream_t st) {
    const int64_t n = nu * nv;
    hipLaunchKernelGGL(test_columns_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, cls, total, nu, nv, su,
                       sv, sa, tca, tnca, alpha_nz, cols);
    return hipGetLastError();
}

}  // namespace vr
