// vr_api.cpp -- C-ABI (include/vr_api.h) over the HIP kernels: the drop-in replacement of the
// reference's myCUDAspace wrappers (kernel.h:15-75, kernel.cu:876-1279).
//
// A vr_ctx owns, on ONE GPU:
//   vol        float32 volume, x-major (kept for re-classification when the TF changes)
//   cls_vrc    uint8 class per voxel for VRC      (TF of max(0,v)/(float)(int)cal_max)
//   cls_test   uint8 class per voxel for TEST     (TF of (float)(v/cal_max)), built on first use
//   maps       3 x 2^D int32 leaf -> voxel maps (the octree leaf grid in closed form)
//   occ        macro-cell occupancy bitmask over the leaf grid (ESS)
//   tf_rgba    class colours; tf_lohi interval bounds
//   work/order cached per (W, H, tiling) work-tile list and XCD-aware block order
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <limits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "ctx.h"
#include "vr_march.h"

#pragma clang fp contract(off)

namespace vr {
hipError_t launch_classify(const float*, int64_t, float, double, const float*, const float*, int, uint8_t*,
                           uint8_t*, const int64_t*, int64_t, int64_t, hipStream_t);
hipError_t launch_occupancy(const uint8_t*, const int32_t*, int, int, int, const int64_t*, const int64_t*,
                            const int64_t*, const uint8_t*, int, unsigned long long*, hipStream_t);
hipError_t launch_vrc_march(const VrcFrame&, const WorkTile*, const int32_t*, int, const uint8_t*,
                            const int32_t*, const int64_t*, const uint32_t*, const float4*, int, float4*,
                            hipStream_t, int, const float*, const int32_t*, const unsigned long long*,
                            const uint8_t*, const int32_t*, int32_t*, unsigned long long*);
size_t vrc_axis1_table_bytes(const VrcFrame&, int);
int vrc_batch_of(const VrcFrame&, int);
hipError_t launch_vrc_stats(const VrcFrame&, const WorkTile*, const int32_t*, int, const uint8_t*, const int32_t*,
                            const uint32_t*, const float4*, int, float4*, unsigned long long*, hipStream_t,
                            const unsigned long long*, const uint8_t*, const int32_t*);
hipError_t launch_occ_columns(const unsigned long long*, int, unsigned long long*, hipStream_t);
hipError_t launch_leaf_columns(const unsigned long long*, int, int, unsigned long long*, hipStream_t);
hipError_t launch_cell_dist(const unsigned long long*, int, int, uint8_t*, uint8_t*, uint8_t**, hipStream_t);
hipError_t launch_test_corners(const uint8_t*, int64_t, int64_t, int64_t, int64_t, const int32_t*, int, uint8_t*,
                               hipStream_t);
hipError_t launch_pack_classes(const uint8_t*, int64_t, int, uint8_t*, hipStream_t);
hipError_t launch_test_faces(const uint8_t*, int64_t, int64_t, int64_t, int32_t*, hipStream_t);
hipError_t launch_test_columns(const uint8_t*, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int, int,
                               const uint8_t*, unsigned long long*, hipStream_t);
hipError_t launch_vrc_count(const VrcFrame&, const WorkTile*, int, const int32_t*, unsigned long long*,
                            hipStream_t);
hipError_t launch_test_march(const TestFrame&, const WorkTile*, const int32_t*, int, const uint8_t*, const float4*, int,
                             const uint32_t*, float4*, hipStream_t, const unsigned long long*, const uint8_t*,
                             const int32_t*, unsigned long long*, const int32_t*, int);
hipError_t launch_test_occupancy(const uint8_t*, int64_t, int64_t, int64_t, int, int, int, int, const uint8_t*,
                                 unsigned long long*, hipStream_t);
hipError_t launch_assemble(int, int, int, int, int, int, const float4*, float4*, int, hipStream_t);
hipError_t launch_assemble_list(int, int, int, int, const int32_t*, const float4*, float4, float4*, int, hipStream_t,
                                int n_frames = 1);
hipError_t launch_worklist(int, int, int, int, int, int, int, WorkTile*, const WlCull&, int, hipStream_t);
void worklist_size(int, int, int, int, int, int, int*, int*, int);
hipError_t launch_normals(const float*, int64_t, int64_t, int64_t, float4*, hipStream_t);
hipError_t launch_synthetic(float*, int64_t, int64_t, int64_t, uint64_t, hipStream_t);
hipError_t launch_egress(const float4*, uint8_t*, int, int, int, hipStream_t);
hipError_t launch_point(const float*, int64_t, int64_t, int64_t, double, const float*, const float*, int,
                        const float4*, float*, hipStream_t);
}  // namespace vr

using namespace vr;

namespace vr {
thread_local std::string g_last_hip_error;
}  // namespace vr

namespace vr {

int tf_index(const std::vector<vr_tf_interval>& tf, float v) {
    int r = 0;
    for (int i = 0; i < (int)tf.size(); ++i)
        if (v >= tf[i].lo && v <= tf[i].hi) r = i;
    return r;
}

void set_device(vr_ctx* c) { hip_check(hipSetDevice(c->device)); }

size_t checked_count(int64_t d1, int64_t d2, int64_t d3) {
    if (d1 <= 0 || d2 <= 0 || d3 <= 0) throw Error(VR_EINVAL, "volume dims must be positive");
    const int64_t lim = INT64_MAX / 16;   // float32 bytes and the class volume's bricked padding stay in int64
    if (d1 > lim / d2 || d1 * d2 > lim / d3) throw Error(VR_ERANGE, "volume dims overflow");
    return (size_t)(d1 * d2 * d3);
}

void reap_retired(vr_ctx* c, bool wait) {
    for (size_t i = 0; i < c->retired.size();) {
        Retired& r = c->retired[i];
        hipError_t q = hipSuccess;
        for (hipEvent_t e : r.ev) {
            const hipError_t qe = wait ? hipEventSynchronize(e) : hipEventQuery(e);
            if (qe != hipSuccess) { q = qe; break; }
        }
        if (q == hipErrorNotReady) { ++i; continue; }
        for (hipEvent_t e : r.ev) (void)hipEventDestroy(e);
        c->retired.erase(c->retired.begin() + (std::ptrdiff_t)i);   // frees the buffers
        if (q != hipSuccess) hip_check(q);
    }
}

void retire_buffers(vr_ctx* c, const std::vector<DevBuf*>& bufs, std::vector<std::vector<int32_t>>* hosts) {
    reap_retired(c, false);
    Retired r;
    std::vector<hipStream_t> st{c->stream};
    for (hipStream_t s : {c->batch_main, c->aux_stream[0], c->aux_stream[1], c->aux_stream[2]})
        if (s && std::find(st.begin(), st.end(), s) == st.end()) st.push_back(s);
    try {
        for (hipStream_t s : st) {
            hipEvent_t e;
            hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            r.ev.push_back(e);
            hip_check(hipEventRecord(e, s));
        }
    } catch (...) {
        for (hipEvent_t e : r.ev) (void)hipEventDestroy(e);
        throw;
    }
    for (DevBuf* b : bufs) {
        r.bufs.emplace_back(new DevBuf);
        r.bufs.back()->swap(*b);
    }
    if (hosts) r.hosts = std::move(*hosts);
    c->retired.push_back(std::move(r));
}

// The per-stream caches -- AXIS1 view tables (axtab), whole-frame work lists (frame_lists), TEST
// axis tables (ztabs) -- of stream `only`, or of every stream but the current one when `only` is
// null (the current stream's entries may be in use by the render call under way): retired behind
// the work queued so far and erased.  No wait on the cached streams themselves: a handle may be dead
// (the context's own stream released by vr_set_stream, or a caller's stream destroyed since).  The
// retire events sit on the context's live streams, which vr_set_stream's switch event ordered after
// everything queued on every earlier stream.
void retire_stream_caches(vr_ctx* c, const hipStream_t* only) {
    std::vector<DevBuf*> v;
    std::vector<std::vector<int32_t>> hosts;
    auto pick = [&](hipStream_t s) { return only ? s == *only : s != c->stream; };
    for (auto& kv : c->axtab)
        if (pick(kv.first)) v.push_back(&kv.second.buf);
    for (auto& kv : c->frame_lists)
        if (pick(kv.first)) v.push_back(&kv.second.wc.work);
    for (auto& kv : c->ztabs)
        if (pick(kv.first)) {
            v.push_back(&kv.second.buf);
            hosts.push_back(std::move(kv.second.host));
        }
    retire_buffers(c, v, &hosts);
    auto drop = [&](auto& m) {
        for (auto it = m.begin(); it != m.end();) it = pick(it->first) ? m.erase(it) : std::next(it);
    };
    drop(c->axtab);
    drop(c->frame_lists);
    drop(c->ztabs);
}
// per-stream caches kept for at most this many streams (then the other streams' are retired)
constexpr size_t kMaxStreamCaches = 8;

// every buffer of the work-list cache, retired behind the work queued so far; the cache is emptied
void retire_work_cache(vr_ctx* c) {
    std::vector<DevBuf*> v;
    for (auto& kv : c->work_cache) v.push_back(&kv.second->work);
    retire_buffers(c, v);
    c->work_cache.clear();
}

void retire_slot_maps(vr_ctx* c) {
    std::vector<DevBuf*> v;
    for (auto& kv : c->slot_maps) v.push_back(kv.second.get());
    retire_buffers(c, v);
    c->slot_maps.clear();
}

// Class bits per voxel the current TF needs (vr_options.class_bits, 0 = auto: the fewest that hold
// every class, 2 / 4 / 8; a forced width below that is raised to it).
int required_cbits(const vr_ctx* c) {
    const int n = (int)c->tf.size();
    const int need = n <= 4 ? 2 : (n <= 16 ? 4 : 8);
    const int want = c->opt.class_bits == 0 ? need : (int)c->opt.class_bits;
    return std::max(need, want);
}

// The separable brick layout of a d1 x d2 x d3 volume: slots in bricks of b voxels per axis, x-major
// over bricks; lay = Fx (d1) | Fy (d2) | Fz (d3), offset(x, y, z) = Fx[x] + Fy[y] + Fz[z] in slots.
// Returns the slot count (voxels and brick padding).
int64_t brick_layout(const int64_t dd[3], const int b[3], std::vector<int64_t>& lay) {
    int64_t nb[3];
    for (int a = 0; a < 3; ++a) nb[a] = (dd[a] + b[a] - 1) / b[a];
    const int64_t bs = (int64_t)b[0] * b[1] * b[2];
    lay.resize((size_t)(dd[0] + dd[1] + dd[2]));
    for (int64_t x = 0; x < dd[0]; ++x) lay[x] = (x / b[0]) * (nb[1] * nb[2] * bs) + (x % b[0]) * (b[1] * b[2]);
    for (int64_t y = 0; y < dd[1]; ++y) lay[dd[0] + y] = (y / b[1]) * (nb[2] * bs) + (y % b[1]) * b[2];
    for (int64_t z = 0; z < dd[2]; ++z) lay[dd[0] + dd[1] + z] = (z / b[2]) * bs + (z % b[2]);
    return nb[0] * nb[1] * nb[2] * bs;
}

// Premultiplied leaf maps: leaf -> Fx[vx], Fy[vy], Fz[vz] (-1 outside) times u units per slot, so a
// sample's class offset is mx + my + mz; x64: the x offsets in 64 bits (IDX64 volumes)
void upload_pmaps(const vr_ctx* c, const std::vector<int64_t>& lay, int64_t u, bool x64, vr::DevBuf& pmaps,
                  vr::DevBuf* pmapx64, vr::DevBuf* pmaps_pad) {
    const int nl = c->oct.nleaf;
    const int64_t d1 = c->d[0], d2 = c->d[1];
    std::vector<int32_t> pm((size_t)3 * nl);
    std::vector<int64_t> px(x64 ? (size_t)nl : 0);
    for (int i = 0; i < nl; ++i) {
        const int32_t vx = c->oct.maps[i], vy = c->oct.maps[nl + i], vz = c->oct.maps[2 * nl + i];
        const int64_t ox = vx < 0 ? -1 : lay[vx] * u;
        if (x64) px[i] = ox; else pm[i] = (int32_t)ox;
        pm[nl + i] = vy < 0 ? -1 : (int32_t)(lay[d1 + vy] * u);
        pm[2 * nl + i] = vz < 0 ? -1 : (int32_t)(lay[d1 + d2 + vz] * u);
    }
    pmaps.ensure(pm.size() * sizeof(int32_t));
    hip_check(hipMemcpy(pmaps.p, pm.data(), pm.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    if (pmaps_pad && !x64) {   // general views' staging copy: kMapOut outside the dataset and in the padding
        const size_t span = (size_t)nl + 2 * kMapPadMax;
        std::vector<int32_t> pp(3 * span, kMapOut);
        for (int a = 0; a < 3; ++a)
            for (int i = 0; i < nl; ++i) {
                const int32_t v = pm[(size_t)a * nl + i];
                pp[a * span + kMapPadMax + i] = v < 0 ? kMapOut : v;
            }
        pmaps_pad->ensure(pp.size() * sizeof(int32_t));
        hip_check(hipMemcpy(pmaps_pad->p, pp.data(), pp.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    } else if (pmaps_pad) {
        pmaps_pad->reset();
    }
    if (x64) {
        pmapx64->ensure(px.size() * sizeof(int64_t));
        hip_check(hipMemcpy(pmapx64->p, px.data(), px.size() * sizeof(int64_t), hipMemcpyHostToDevice));
    }
}

// The class-volume layout for cbits bits per class (brick_layout); the default brick is 128 B at
// every width (4 x 4 x 8 slots at 8 bits, 4 x 8 x 8 at 4, 8 x 8 x 8 at 2).  The march addresses
// classes in bits when cbits < 8 (byte = o >> 3, the class at bit o & 7) and in bytes at 8 bits;
// the premultiplied leaf maps hold those units.  Volumes whose offsets would pass 2^31 - 64 units
// keep the x offsets in 64 bits (IDX64), in the same units.  A compact 32-bit volume also gets the
// general views' byte-per-class copy's layout (vr_ctx::gen) in the options' brick.
void build_layout(vr_ctx* c, int cbits) {
    const int64_t dd[3] = {c->d[0], c->d[1], c->d[2]};
    const bool def_brick = c->opt.brick[0] == 4 && c->opt.brick[1] == 4 && c->opt.brick[2] == 8;
    for (int a = 0; a < 3; ++a) c->brick[a] = c->opt.brick[a];
    if (def_brick && cbits == 4) c->brick[1] = 8;
    if (def_brick && cbits == 2) { c->brick[0] = 8; c->brick[1] = 8; }
    c->cls_slots = brick_layout(dd, c->brick, c->lay);
    const int64_t units = cbits < 8 ? c->cls_slots * cbits : c->cls_slots;   // bits or bytes
    // (64 units short of 2^31: the axis-aligned march's table markers rely on the margin)
    c->idx64 = units > ((int64_t)1 << 31) - 64 || c->opt.force_idx64 != 0;
    c->cbits = cbits;
    c->cls_bytes = (c->cls_slots * cbits + 7) / 8;
    c->layout.ensure(c->lay.size() * sizeof(int64_t));
    hip_check(hipMemcpy(c->layout.p, c->lay.data(), c->lay.size() * sizeof(int64_t), hipMemcpyHostToDevice));
    upload_pmaps(c, c->lay, cbits < 8 ? cbits : 1, c->idx64, c->pmaps, &c->pmapx64, &c->pmaps_pad);
    c->gen = cbits < 8 && !c->idx64;
    if (c->gen) {
        c->gen_bytes = brick_layout(dd, c->opt.brick, c->lay_gen);   // (< 2^31 / cbits bytes)
        c->layout_gen.ensure(c->lay_gen.size() * sizeof(int64_t));
        hip_check(hipMemcpy(c->layout_gen.p, c->lay_gen.data(), c->lay_gen.size() * sizeof(int64_t),
                            hipMemcpyHostToDevice));
        upload_pmaps(c, c->lay_gen, 1, false, c->pmaps_gen, nullptr, &c->pmaps_gen_pad);
    } else {
        c->gen_bytes = 0;
        c->lay_gen.clear();
        c->cls_gen.reset();
        c->layout_gen.reset();
        c->pmaps_gen.reset();
        c->pmaps_gen_pad.reset();
    }
}

// (Re)classify the volume and rebuild the occupancy pyramid for the current TF.
void classify(vr_ctx* c, bool need_test) {
    const int n_tf = (int)c->tf.size();
    std::vector<float> lohi(2 * n_tf);
    std::vector<float4> rgba(n_tf);
    std::vector<uint8_t> anz(kMaxTf, 0);
    for (int i = 0; i < n_tf; ++i) {
        lohi[i] = c->tf[i].lo;
        lohi[n_tf + i] = c->tf[i].hi;
        rgba[i] = make_float4(c->tf[i].rgba[0], c->tf[i].rgba[1], c->tf[i].rgba[2], c->tf[i].rgba[3]);
        anz[i] = c->tf[i].rgba[3] != 0.0f;
    }
    c->tf_lohi.ensure(lohi.size() * sizeof(float));
    c->tf_rgba.ensure(kMaxTf * sizeof(float4));
    c->alpha_nz.ensure(kMaxTf);
    hip_check(hipMemcpyAsync(c->tf_lohi.p, lohi.data(), lohi.size() * sizeof(float), hipMemcpyHostToDevice, c->stream));
    hip_check(hipMemcpyAsync(c->tf_rgba.p, rgba.data(), rgba.size() * sizeof(float4), hipMemcpyHostToDevice, c->stream));
    hip_check(hipMemcpyAsync(c->alpha_nz.p, anz.data(), kMaxTf, hipMemcpyHostToDevice, c->stream));
    // class of the value 0 (outside the cube / dataset): VRC 0 / (float)(int)cal_max, TEST 0 / cal_max
    c->cls0_vrc = tf_index(c->tf, 0.0f / (float)c->max_intensity);
    c->cls0_test = tf_index(c->tf, (float)(0.0 / c->cal_max));
    c->zero_transparent = c->tf[c->cls0_vrc].rgba[3] == 0.0f && c->tf[c->cls0_test].rgba[3] == 0.0f;
    const int64_t n = c->d[0] * c->d[1] * c->d[2];
    const int cb = required_cbits(c);
    if (cb != c->cbits) {   // a TF with more classes than the layout holds (or an option change)
        ctx_sync(c, c->stream);   // (the layout tables and leaf maps are replaced under queued launches)
        build_layout(c, cb);
        std::vector<DevBuf*> v;   // published view tables hold offsets of the old layout
        for (auto& kv : c->axtab) v.push_back(&kv.second.buf);
        retire_buffers(c, v);
        c->axtab.clear();
    }
    // the classes one byte per slot (cls8: the occupancy pass reads them), packed into cls_vrc at
    // cbits < 8 (8 bits: cls_vrc is that volume itself)
    DevBuf& c8 = c->cbits < 8 ? c->cls8 : c->cls_vrc;
    if (c->cbits == 8) c->cls8.reset();
    c8.ensure((size_t)c->cls_slots);
    hip_check(hipMemsetAsync(c8.p, c->cls0_vrc, (size_t)c->cls_slots, c->stream));
    uint8_t* test_out = nullptr;
    if (need_test) {
        c->cls_test.ensure((size_t)n + kClsPad);
        hip_check(hipMemsetAsync(c->cls_test.as<uint8_t>() + n, 0, kClsPad, c->stream));
        test_out = c->cls_test.as<uint8_t>();
    }
    hip_check(launch_classify(c->vol.as<float>(), n, (float)c->max_intensity, c->cal_max, c->tf_lohi.as<float>(),
                              c->tf_lohi.as<float>() + n_tf, n_tf, c8.as<uint8_t>(), test_out,
                              c->layout.as<int64_t>(), c->d[1], c->d[2], c->stream));
    group_mark(c);   // (multi-GPU parts: progress for the polled waits' deadline, vr_multi.cpp)
    if (c->cbits < 8) {
        c->cls_vrc.ensure((size_t)c->cls_bytes + 16);
        hip_check(launch_pack_classes(c8.as<uint8_t>(), c->cls_slots, c->cbits, c->cls_vrc.as<uint8_t>(), c->stream));
    }
    if (c->gen) {   // the general views' byte-per-class copy (its own brick layout)
        c->cls_gen.ensure((size_t)c->gen_bytes);
        hip_check(hipMemsetAsync(c->cls_gen.p, c->cls0_vrc, (size_t)c->gen_bytes, c->stream));
        hip_check(launch_classify(c->vol.as<float>(), n, (float)c->max_intensity, c->cal_max, c->tf_lohi.as<float>(),
                                  c->tf_lohi.as<float>() + n_tf, n_tf, c->cls_gen.as<uint8_t>(), nullptr,
                                  c->layout_gen.as<int64_t>(), c->d[1], c->d[2], c->stream));
        group_mark(c);
    }
    c->cls_test_valid = need_test;
    // occupancy over the leaf grid
    const int64_t ncells = (int64_t)c->ncell * c->ncell * c->ncell;
    c->occ.ensure((size_t)((ncells + 63) / 64) * 8);
    const int64_t* L = c->layout.as<int64_t>();
    hip_check(launch_occupancy(c8.as<uint8_t>(), c->maps.as<int32_t>(), c->oct.nleaf, c->cb_shift, c->ncell,
                               L, L + c->d[0], L + c->d[0] + c->d[1], c->alpha_nz.as<uint8_t>(), c->cls0_vrc,
                               c->occ.as<unsigned long long>(), c->stream));
    group_mark(c);
    c->occ_cols.ensure((size_t)3 * c->ncell * c->ncell * 8);
    hip_check(launch_occ_columns(c->occ.as<unsigned long long>(), c->ncell, c->occ_cols.as<unsigned long long>(),
                                 c->stream));
    // axis views: one column mask per LEAF column (the exact set a ray of the view crosses) from the
    // occupancy of single leaves; up to kLeafColsMax leaves per axis (2048^3 bits = 1 GB transient)
    c->leafcols = c->oct.nleaf <= kLeafColsMax && c->opt.leaf_columns != 0;
    if (c->leafcols) {
        const int nl = c->oct.nleaf;
        DevBuf locc;
        locc.ensure((size_t)(((int64_t)nl * nl * nl + 63) / 64) * 8);
        hip_check(launch_occupancy(c8.as<uint8_t>(), c->maps.as<int32_t>(), nl, 0, nl, L, L + c->d[0],
                                   L + c->d[0] + c->d[1], c->alpha_nz.as<uint8_t>(), c->cls0_vrc,
                                   locc.as<unsigned long long>(), c->stream));
        c->occ_leafcols.ensure((size_t)3 * nl * nl * 8);
        hip_check(launch_leaf_columns(locc.as<unsigned long long>(), nl, c->cb_shift,
                                      c->occ_leafcols.as<unsigned long long>(), c->stream));
        ctx_sync(c, c->stream);   // (locc is freed on return)
    }
    {   // Chebyshev cell distances (capped; two ping-pong halves of one buffer)
        const size_t nc = (size_t)ncells;
        c->cdist.ensure(2 * nc);
        uint8_t* res = nullptr;
        hip_check(launch_cell_dist(c->occ.as<unsigned long long>(), c->ncell, kCellDistCap, c->cdist.as<uint8_t>(),
                                   c->cdist.as<uint8_t>() + nc, &res, c->stream));
        c->cdist_p = res;
    }
    {   // bounding range of the occupied macro cells (screen-space culling tightens to it)
        std::vector<unsigned long long> h((size_t)((ncells + 63) / 64));
        hip_check(hipMemcpyAsync(h.data(), c->occ.p, h.size() * 8, hipMemcpyDeviceToHost, c->stream));
        ctx_sync(c, c->stream);
        for (int a = 0; a < 3; ++a) { c->occ_lo[a] = c->ncell; c->occ_hi[a] = -1; }
        const int64_t nc = c->ncell;
        const size_t side = (size_t)nc + 1;
        for (int a = 0; a < 3; ++a) c->col_sat[a].assign(side * side, 0);
        for (int64_t cell = 0; cell < ncells; ++cell)
            if ((h[(size_t)(cell >> 6)] >> (cell & 63)) & 1ull) {
                const int cc[3] = {(int)(cell / (nc * nc)), (int)((cell / nc) % nc), (int)(cell % nc)};
                for (int a = 0; a < 3; ++a) {
                    c->occ_lo[a] = std::min(c->occ_lo[a], cc[a]);
                    c->occ_hi[a] = std::max(c->occ_hi[a], cc[a]);
                    const int u = cc[a == 0 ? 1 : 0], v = cc[a == 2 ? 1 : 2];
                    c->col_sat[a][(size_t)(u + 1) * side + (size_t)(v + 1)] = 1;   // the column along a
                }
            }
        c->sc_shift = 0;
        while ((c->ncell >> c->sc_shift) > 16) ++c->sc_shift;
        c->nsc = (c->ncell + (1 << c->sc_shift) - 1) >> c->sc_shift;
        c->socc.assign((size_t)c->nsc * c->nsc * c->nsc, 0);
        for (int64_t cell = 0; cell < ncells; ++cell)
            if ((h[(size_t)(cell >> 6)] >> (cell & 63)) & 1ull) {
                const int sx = (int)(cell / (nc * nc)) >> c->sc_shift, sy = (int)((cell / nc) % nc) >> c->sc_shift,
                          sz = (int)(cell % nc) >> c->sc_shift;
                c->socc[((size_t)sx * c->nsc + sy) * c->nsc + sz] = 1;
            }
        c->vis_cache.clear();
        for (int a = 0; a < 3; ++a)   // prefix sums: sat[u][v] = occupied columns in [0, u) x [0, v)
            for (size_t u = 1; u < side; ++u)
                for (size_t v = 1; v < side; ++v)
                    c->col_sat[a][u * side + v] += c->col_sat[a][(u - 1) * side + v] + c->col_sat[a][u * side + v - 1] -
                                                   c->col_sat[a][(u - 1) * side + v - 1];
        // the device copy for worklist_kernel's cull (stream-ordered after every queued list build)
        std::vector<int32_t> all;
        for (int a = 0; a < 3; ++a) all.insert(all.end(), c->col_sat[a].begin(), c->col_sat[a].end());
        c->col_sat_dev.ensure(all.size() * sizeof(int32_t));
        hip_check(hipMemcpyAsync(c->col_sat_dev.p, all.data(), all.size() * sizeof(int32_t), hipMemcpyHostToDevice,
                                 c->stream));
        ctx_sync(c, c->stream);   // (all is a host temporary)
        ++c->sat_gen;
    }
    if (need_test) {   // TEST macro cells: 8^3 voxels, coarser until the bitmask is <= 2^18 bits
        c->tcb = 3;
        auto nc = [&](int a) { return (int)((c->d[a] + (1 << c->tcb) - 1) >> c->tcb); };
        while ((int64_t)nc(0) * nc(1) * nc(2) > (1 << 18)) ++c->tcb;
        for (int a = 0; a < 3; ++a) c->tnc[a] = nc(a);
        const int64_t tcells = (int64_t)c->tnc[0] * c->tnc[1] * c->tnc[2];
        c->occ_test.ensure((size_t)((tcells + 63) / 64) * 8);
        // the faces' classes (TestFrame.lin): read back after the sync at the end of classify
        c->faces_flag.ensure(sizeof(int32_t));
        hip_check(hipMemsetAsync(c->faces_flag.p, 0, sizeof(int32_t), c->stream));
        hip_check(launch_test_faces(c->cls_test.as<uint8_t>(), c->d[0], c->d[1], c->d[2], c->faces_flag.as<int32_t>(),
                                    c->stream));
        hip_check(hipMemcpyAsync(&c->test_faces_dirty, c->faces_flag.p, sizeof(int32_t), hipMemcpyDeviceToHost,
                                 c->stream));
        hip_check(launch_test_occupancy(c->cls_test.as<uint8_t>(), c->d[0], c->d[1], c->d[2], c->tcb, c->tnc[0],
                                        c->tnc[1], c->tnc[2], c->alpha_nz.as<uint8_t>(),
                                        c->occ_test.as<unsigned long long>(), c->stream));
        // general views: the corner volume (one gather per sample), when its offsets fit 32 bits.
        // vr_options.test_corners 0: per voxel the 8 corner classes at the TF's class width (16 bits
        // for <= 4 intervals, 32 for <= 16, else 64), x-major; 1: 64 bits per voxel, x-major (round
        // 4); 2: none; 3: the TF's class width in 4 x 4 x 4-voxel bricks (a wave's rays share a
        // brick's 128-512 B across all three axes)
        {
            const int64_t total = c->d[0] * c->d[1] * c->d[2];
            const int nt = (int)c->tf.size();
            const int mode = c->opt.test_corners;
            const int cb = mode == 1 ? 8 : (nt <= 4 ? 2 : (nt <= 16 ? 4 : 8));
            c->tcv = 0;
            c->tcv_bytes = 0;
            if ((mode == 0 || mode == 1) && total * cb <= ((int64_t)1 << 31) - 64) {
                c->tcc.ensure((size_t)(total * cb));
                hip_check(launch_test_corners(c->cls_test.as<uint8_t>(), total, c->d[0], c->d[1], c->d[2], nullptr, cb,
                                              c->tcc.as<uint8_t>(), c->stream));
                c->tcv = 16 + cb;
                c->tcv_bytes = total * cb;
            } else if (mode == 3) {
                const int64_t dd[3] = {c->d[0], c->d[1], c->d[2]};
                const int b4[3] = {4, 4, 4};
                std::vector<int64_t> lay;
                const int64_t bytes = brick_layout(dd, b4, lay) * cb;   // cb bits x 8 corners = cb bytes
                if (bytes <= ((int64_t)1 << 31) - 64) {
                    std::vector<int32_t> l32(lay.size());
                    for (size_t i = 0; i < lay.size(); ++i) l32[i] = (int32_t)(lay[i] * cb);
                    c->tcc_lay.ensure(l32.size() * sizeof(int32_t));
                    hip_check(hipMemcpyAsync(c->tcc_lay.p, l32.data(), l32.size() * sizeof(int32_t),
                                             hipMemcpyHostToDevice, c->stream));
                    c->tcc.ensure((size_t)bytes);
                    hip_check(hipMemsetAsync(c->tcc.p, 0, (size_t)bytes, c->stream));   // (brick padding)
                    hip_check(launch_test_corners(c->cls_test.as<uint8_t>(), total, c->d[0], c->d[1], c->d[2],
                                                  c->tcc_lay.as<int32_t>(), cb, c->tcc.as<uint8_t>(), c->stream));
                    ctx_sync(c, c->stream);   // (l32 is a host temporary)
                    c->tcv = cb;
                    c->tcv_bytes = bytes;
                }
            }
            if (!c->tcv) {
                c->tcc.reset();
                c->tcc_lay.reset();
            }
            group_mark(c);
        }
        // axis views: per march axis a, occupied cells (tca voxels, at most 64) per corner line of
        // the two other axes, the three tables back to back
        {
            const int64_t d[3] = {c->d[0], c->d[1], c->d[2]};
            const int64_t st[3] = {d[1] * d[2], d[2], 1};   // flat-index strides
            int64_t off = 0;
            for (int a = 0; a < 3; ++a) {
                const int u = a == 0 ? 1 : 0, v = a == 2 ? 1 : 2;
                c->tca[a] = (int)std::max<int64_t>(1, (d[a] + 63) / 64);
                c->tnca[a] = (int)((d[a] + c->tca[a] - 1) / c->tca[a]);
                c->tcol_pitch[a] = (int)(d[v] + 2);
                c->tcol_base[a] = off;
                off += (d[u] + 2) * (d[v] + 2);
            }
            c->tcol.ensure((size_t)off * 8);
            for (int a = 0; a < 3; ++a) {
                const int u = a == 0 ? 1 : 0, v = a == 2 ? 1 : 2;
                hip_check(launch_test_columns(c->cls_test.as<uint8_t>(), d[0] * d[1] * d[2], d[u] + 2, d[v] + 2, st[u],
                                              st[v], st[a], c->tca[a], c->tnca[a], c->alpha_nz.as<uint8_t>(),
                                              c->tcol.as<unsigned long long>() + c->tcol_base[a], c->stream));
            }
        }
    }
    ctx_sync(c, c->stream);
    c->cls8.reset();   // (the one-byte classes are only the occupancy pass's input: C5 holds 8.6 GB of them)
}

void set_tf(vr_ctx* c, const vr_tf_interval* tf, int32_t n_tf) {
    if (!tf || n_tf <= 0 || n_tf > kMaxTf) throw Error(VR_EINVAL, "transfer function: need 1..256 intervals");
    c->tf.assign(tf, tf + n_tf);
}

void check_options(const vr_options& o) {
    for (int a = 0; a < 3; ++a)
        if (o.brick[a] <= 0 || o.brick[a] > 64) throw Error(VR_EINVAL, "vr_options: brick sizes must be 1..64");
    if (o.batch != 0 && o.batch != 8 && o.batch != 16) throw Error(VR_EINVAL, "vr_options: batch must be 0, 8 or 16");
    if (o.work_order < 0 || o.work_order > 2) throw Error(VR_EINVAL, "vr_options: work_order must be 0..2");
    if (o.persist_wgs < 0 || o.persist_wgs > 32) throw Error(VR_EINVAL, "vr_options: persist_wgs must be 0..32");
    if (o.cell_shift < -1 || o.cell_shift > 16) throw Error(VR_EINVAL, "vr_options: cell_shift must be -1..16");
    if (o.comm_timeout_ms < 0) throw Error(VR_EINVAL, "vr_options: comm_timeout_ms must be >= 0");
    if (o.class_bits != 0 && o.class_bits != 2 && o.class_bits != 4 && o.class_bits != 8)
        throw Error(VR_EINVAL, "vr_options: class_bits must be 0, 2, 4 or 8");
    if (o.run_words < 0 || o.run_words > 2) throw Error(VR_EINVAL, "vr_options: run_words must be 0, 1 or 2");
    if (o.frames_in_flight < 0 || o.frames_in_flight > 3)
        throw Error(VR_EINVAL, "vr_options: frames_in_flight must be 0..3");
    if (o.table_split != 0 && o.table_split != 1) throw Error(VR_EINVAL, "vr_options: table_split must be 0 or 1");
    if (o.test_corners < 0 || o.test_corners > 3) throw Error(VR_EINVAL, "vr_options: test_corners must be 0..3");
    if (o.leaf_columns < 0 || o.leaf_columns > 1) throw Error(VR_EINVAL, "vr_options: leaf_columns must be 0 or 1");
    if (o.farm_tile <= 0 || o.farm_tile % kWgRaysX || o.farm_tile > 4096)
        throw Error(VR_EINVAL, "vr_options: farm_tile must be a positive multiple of 16");
    if (!(o.farm_rank0_weight > 0.0f && o.farm_rank0_weight <= 1e9f))
        throw Error(VR_EINVAL, "vr_options: farm_rank0_weight must be positive");
}

// render-time options: safe to change between frames (cached work lists depend on the order)
void apply_render_options(vr_ctx* c, const vr_options& o) {
    if (c->order_mode != o.work_order) {   // (cached lists may be in flight: retired, not freed)
        set_device(c);
        retire_work_cache(c);
    }
    c->batch = o.batch;
    c->occ_lds = o.occ_lds != 0;
    c->axis1_ok = o.axis_table != 0;
    c->persist_wgs = o.persist_wgs;
    c->order_mode = o.work_order;
    c->cull = o.cull < 0 ? 0 : o.cull;
    c->tab_reuse = o.view_table_reuse != 0;
    c->test_axz = o.test_plane_march != 0;
    c->opt = o;
}

vr_ctx* create_common(const float* voxels, bool on_device, int64_t d1, int64_t d2, int64_t d3, double cal_max,
                      const vr_tf_interval* tf, int32_t n_tf, int32_t device, const vr_options* opt_in,
                      DevBuf* adopt_vol) {
    if (!voxels && !adopt_vol) throw Error(VR_EINVAL, "vr_create: bad volume");
    (void)checked_count(d1, d2, d3);
    vr_options opt;
    vr_options_default(&opt);
    if (opt_in) opt = *opt_in;
    check_options(opt);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) throw Error(VR_ENODEV, "vr_create: no GPU");
    if (device < 0 || device >= ndev) throw Error(VR_ENODEV, "vr_create: bad device index");
    std::unique_ptr<vr_ctx> c(new vr_ctx);
    c->device = device;
    set_device(c.get());
    hip_check(hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking));
    c->stream = c->own_stream;
    c->d[0] = d1; c->d[1] = d2; c->d[2] = d3;
    c->cal_max = cal_max;
    c->max_intensity = (int)cal_max;   // kernel.cu:1151 passes double cal_max as int max_intensity
    set_tf(c.get(), tf, n_tf);
    c->oct.build(d1, d2, d3);
    const int D = (int)c->oct.maximum_depth;
    // macro cells of 4 leaves (measured: 4.6 % faster than 8 at C3), coarser for deep trees so a
    // cell column fits the uint64 occupancy mask of the axis-aligned march (<= 64 cells per axis)
    c->cb_shift = D <= 2 ? D : std::max(2, D - 6);
    if (opt.cell_shift >= 0) c->cb_shift = std::max(std::max(0, D - 6), std::min(D, (int)opt.cell_shift));
    c->ncell = c->oct.nleaf >> c->cb_shift;
    const int64_t n = d1 * d2 * d3;
    if (adopt_vol) {   // a device buffer of this GPU holding the volume (multi-GPU broadcast target)
        if (adopt_vol->bytes < (size_t)n * sizeof(float)) throw Error(VR_EINVAL, "vr_create: adopted volume too small");
        c->vol.swap(*adopt_vol);
    } else {
        c->vol.ensure((size_t)n * sizeof(float));
        hip_check(hipMemcpyAsync(c->vol.p, voxels, (size_t)n * sizeof(float),
                                 on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, c->stream));
    }
    c->maps.ensure(c->oct.maps.size() * sizeof(int32_t));
    hip_check(hipMemcpyAsync(c->maps.p, c->oct.maps.data(), c->oct.maps.size() * sizeof(int32_t),
                             hipMemcpyHostToDevice, c->stream));
    // layout options (defaults chosen by measurement) and render options
    apply_render_options(c.get(), opt);
    build_layout(c.get(), required_cbits(c.get()));
    c->counter.ensure(64);
    classify(c.get(), false);
    return c.release();
}

// XCD-aware block order of a work list (the permuted list; holes are tiles far off screen).
std::vector<WorkTile> dispatch_order(const vr_ctx* c, const std::vector<WorkTile>& wl, int W, int H) {
    // XCD-aware block order.  Blocks b and b+8 share an XCD under the observed round-robin
    // dispatch (speed only, never correctness), so position 8*j + x of `order` is XCD group x's
    // j-th tile, and each group walks its tiles in screen order (tile columns left to right).
    // order_mode 0 (default): diagonal interleave, work tile (tx, ty) -> group (tx + ty) % 8: every
    // group gets an eighth of every tile column, so the costly centre of the frame is spread over
    // all eight L2s and the groups finish together (against column bands: C2 -4 %, exact -6 %,
    // TEST -7 %, C3 and oblique within 2 %).  order_mode 2: screen bands of tile columns, band k ->
    // group k % 8 (the previous default).  order_mode 1: the reference's camera always looks at
    // the volume centre (myApp.cu:1107), so the costly tiles surround the screen centre; each group
    // gets one of 8 angular sectors walked from the centre outwards.
    std::vector<std::vector<int>> per_xcd(8);
    if (c->order_mode == 0) {
        for (int i = 0; i < (int)wl.size(); ++i)
            per_xcd[(wl[i].x0 / kWgRaysX + wl[i].y0 / kWgRaysY) % 8].push_back(i);
    } else if (c->order_mode == 2) {
        int max_x0 = 0;
        for (auto& w : wl) max_x0 = std::max(max_x0, w.x0);
        const int ncols = max_x0 / kWgRaysX + 1;
        // (bands of 4 tile columns measured worse on general views: VRC oblique +3 %, TEST +2-7 %,
        // although they halve the reads past L2 -- profiles/r5_ab/deal_*.log)
        const int band_cols = std::max(1, ncols / 64);
        for (int i = 0; i < (int)wl.size(); ++i) per_xcd[((wl[i].x0 / kWgRaysX) / band_cols) % 8].push_back(i);
    } else {
        const double cx = 0.5 * W, cy = 0.5 * H;
        std::vector<std::pair<double, int>> key(wl.size());
        std::vector<int> sector(wl.size());
        for (int i = 0; i < (int)wl.size(); ++i) {
            const double dx = wl[i].x0 + 0.5 * kWgRaysX - cx, dy = wl[i].y0 + 0.5 * kWgRaysY - cy;
            const double ang = std::atan2(dy, dx) + M_PI;
            sector[i] = std::min(7, (int)(ang / (2 * M_PI) * 8));
            key[i] = {dx * dx + dy * dy, i};
        }
        std::sort(key.begin(), key.end());
        for (auto& k : key) per_xcd[sector[k.second]].push_back(k.second);
    }
    size_t maxc = 0;
    for (auto& v : per_xcd) maxc = std::max(maxc, v.size());
    std::vector<int32_t> order(8 * maxc, -1);
    for (int x = 0; x < 8; ++x)
        for (size_t j = 0; j < per_xcd[x].size(); ++j) order[8 * j + x] = per_xcd[x][j];
    // drop a trailing all-empty tail
    while (!order.empty() && order.back() < 0) order.pop_back();
    // the work list is stored already permuted into dispatch order (block b reads work[b]: one load,
    // no order[] indirection); holes become tiles far off screen, which every kernel skips
    std::vector<WorkTile> wp(order.size());
    for (size_t b = 0; b < order.size(); ++b)
        wp[b] = order[b] >= 0 ? wl[(size_t)order[b]] : WorkTile{1 << 30, 1 << 30, 0, 0};
    return wp;
}

// Work tiles (16x16 rays) + an XCD-aware block order: work tile (tx, ty) goes to XCD (tx + ty) % 8
// (blocks b and b+8 share an XCD under the observed round-robin dispatch).
// list (tile mode only): render the tiles list[first], list[first + stride], ... instead of the
// tile ids first, first + stride, ... of the whole grid
// rect (whole-frame mode only): march only the 16 x 16 work tiles inside it; the others are
// appended with slot = -1 and the march kernel stores the background for them
WorkCache* work_for(vr_ctx* c, int W, int H, int tile_w, int tile_h, int first, int stride,
                    const std::vector<int32_t>* list = nullptr, const TileRect* rect = nullptr) {
    const bool culled = tile_w == 0 && rect && !rect->all;
    auto key = std::make_tuple(W, H, tile_w, tile_h, first, stride,
                               list ? *list : (culled ? std::vector<int32_t>{-2, rect->tx0, rect->tx1, rect->ty0,
                                                                              rect->ty1}
                                                      : std::vector<int32_t>{-1}));
    auto it = c->work_cache.find(key);
    if (it != c->work_cache.end()) return it->second.get();
    if (c->work_cache.size() > 64) retire_work_cache(c);   // moving cameras: bound the cache
    std::vector<WorkTile> wl, fl;
    if (tile_w == 0) {   // whole frame, work tiles in x-major order
        for (int x0 = 0; x0 < W; x0 += kWgRaysX)
            for (int y0 = 0; y0 < H; y0 += kWgRaysY) {
                const int tx = x0 / kWgRaysX, ty = y0 / kWgRaysY;
                const bool in = !culled || (tx >= rect->tx0 && tx <= rect->tx1 && ty >= rect->ty0 && ty <= rect->ty1);
                (in ? wl : fl).push_back({x0, y0, 0, 0});
            }
    } else {
        const int ntx = (W + tile_w - 1) / tile_w, nty = (H + tile_h - 1) / tile_h;
        const int64_t n_ids = list ? (int64_t)list->size() : (int64_t)ntx * nty;
        int slot = 0;
        for (int64_t i = first; i < n_ids; i += stride, ++slot) {
            const int64_t t = list ? (*list)[(size_t)i] : i;
            const int tx = (int)(t / nty), ty = (int)(t % nty);
            for (int ox = 0; ox < tile_w; ox += kWgRaysX)
                for (int oy = 0; oy < tile_h; oy += kWgRaysY) {
                    const int x0 = tx * tile_w + ox, y0 = ty * tile_h + oy;
                    if (x0 < W && y0 < H) wl.push_back({x0, y0, slot, (ox << 16) | oy});
                }
        }
    }
    std::vector<WorkTile> wp = dispatch_order(c, wl, W, H);
    // culled whole-frame tiles ride at the end of the same launch, marked slot = -1: the march
    // kernel stores the background for them before any staging (one launch per frame)
    const int bg_first = (int)wp.size();
    for (const WorkTile& t : fl) wp.push_back({t.x0, t.y0, -1, 0});
    std::unique_ptr<WorkCache> wc(new WorkCache);
    wc->n_work = (int)wp.size();
    wc->n_blocks = (int)wp.size();
    wc->bg_first = tile_w == 0 ? bg_first : -1;
    wc->work.ensure(std::max<size_t>(1, wp.size()) * sizeof(WorkTile));
    if (!wp.empty())
        hip_check(hipMemcpy(wc->work.p, wp.data(), wp.size() * sizeof(WorkTile), hipMemcpyHostToDevice));
    WorkCache* raw = wc.get();
    c->work_cache[std::move(key)] = std::move(wc);
    return raw;
}

// Whole-frame launch over a subset of the frame's tile x tile user tiles (rank 0 of a multi-GPU
// context): the work tiles of the user tiles in `own` are marched straight into the frame, the work
// tiles of every user tile not in `visible` are background-filled (slot = -1), and the rest (the
// peers' tiles, scattered in after the gather) are not touched.
WorkCache* work_for_subset(vr_ctx* c, int W, int H, int tile, const std::vector<int32_t>& own,
                           const std::vector<int32_t>& visible) {
    std::vector<int32_t> kv(own);
    kv.push_back(-3);
    kv.insert(kv.end(), visible.begin(), visible.end());
    auto key = std::make_tuple(W, H, -tile, -tile, 0, 1, std::move(kv));
    auto it = c->work_cache.find(key);
    if (it != c->work_cache.end()) return it->second.get();
    if (c->work_cache.size() > 64) retire_work_cache(c);
    const int ntx = (W + tile - 1) / tile, nty = (H + tile - 1) / tile;
    std::vector<uint8_t> vis((size_t)ntx * nty, 0);
    for (int32_t t : visible) vis[(size_t)t] = 1;
    std::vector<WorkTile> wl, fl;
    auto add = [&](std::vector<WorkTile>& v, int32_t t, int slot) {
        const int tx = t / nty, ty = t % nty;
        for (int ox = 0; ox < tile; ox += kWgRaysX)
            for (int oy = 0; oy < tile; oy += kWgRaysY) {
                const int x0 = tx * tile + ox, y0 = ty * tile + oy;
                if (x0 < W && y0 < H) v.push_back({x0, y0, slot, 0});
            }
    };
    for (int32_t t : own) add(wl, t, 0);
    for (int32_t t = 0; t < ntx * nty; ++t)
        if (!vis[(size_t)t]) add(fl, t, -1);
    std::vector<WorkTile> wp = dispatch_order(c, wl, W, H);
    wp.insert(wp.end(), fl.begin(), fl.end());
    std::unique_ptr<WorkCache> wc(new WorkCache);
    wc->n_work = wc->n_blocks = (int)wp.size();
    wc->work.ensure(std::max<size_t>(1, wp.size()) * sizeof(WorkTile));
    if (!wp.empty())
        hip_check(hipMemcpy(wc->work.p, wp.data(), wp.size() * sizeof(WorkTile), hipMemcpyHostToDevice));
    WorkCache* raw = wc.get();
    c->work_cache[std::move(key)] = std::move(wc);
    return raw;
}

int cull_axis(const vr_ctx* c, const vr_params* p, const vr_camera* cam);
TestFrame make_test(const vr_ctx* c, const vr_params* p, const vr_camera* cam);

// The whole-frame work list of the default (diagonal) deal, built on the device by worklist_kernel
// on the ctx stream whenever the visible rectangle changes (a moving camera: no host build, no
// upload, no host synchronisation); one buffer per stream, reused in stream order.
WorkCache* frame_list(vr_ctx* c, const vr_params* p, const vr_camera* cam, const TileRect& rect) {
    const int W = p->width, H = p->height;
    const int ntx = (W + kWgRaysX - 1) / kWgRaysX, nty = (H + kWgRaysY - 1) / kWgRaysY;
    int tx0 = 0, tx1 = ntx - 1, ty0 = 0, ty1 = nty - 1;
    if (!rect.all) { tx0 = rect.tx0; tx1 = rect.tx1; ty0 = rect.ty0; ty1 = rect.ty1; }
    if (tx1 < tx0 || ty1 < ty0) { tx0 = ty0 = 0; tx1 = ty1 = -1; }
    // axis-parallel views: work tiles over empty cell columns are marked culled (a function of the
    // camera's two fixed axes too, so those are part of the key)
    WlCull cull{};
    const int ma = cull_axis(c, p, cam);
    // the XCD deal: diagonal, except TEST frames of general views, whose workgroups read the corner
    // volume (14.5 MB at C3, bricked): whole tile columns interleaved over the XCD groups keep each
    // L2's share of it smaller -- 25.5 -> 18.1 MB past L2 per C3 oblique launch at the same frame
    // time, where the diagonal deal's x-major corner volume read 82 MB (profiles/r5_ab/deal_*.log).
    // TEST axis views (test_axis_kernel: no corner volume) are decided by make_test's own test
    // (cull_axis is -1 for every TEST frame, so they took the column deal unmeasured)
#ifndef VR_TEST_AXIS_COLUMN_DEAL
#define VR_TEST_AXIS_COLUMN_DEAL 0
#endif
    const int deal = (p->mode == VR_MODE_TEST && (VR_TEST_AXIS_COLUMN_DEAL || make_test(c, p, cam).axt < 0)) ? 1 : 0;
    std::vector<uint32_t> key = {(uint32_t)W, (uint32_t)H, (uint32_t)tx0, (uint32_t)tx1, (uint32_t)ty0, (uint32_t)ty1,
                                 (uint32_t)ma, (uint32_t)deal};
    if (ma >= 0) {
        const int a0 = ma == 0 ? 1 : 0, a1 = ma == 2 ? 1 : 2;
        const int side = c->ncell + 1;
        cull.sat = c->col_sat_dev.as<int32_t>() + (size_t)ma * side * side;
        cull.side = side;
        cull.cb_shift = c->cb_shift;
        cull.nleaf = (int)c->oct.nleaf;
        cull.W = W; cull.H = H;
        cull.rsw = p->real_screen_width; cull.rsh = p->real_screen_height;
        const int ax[2] = {a0, a1};
        for (int k = 0; k < 2; ++k) {
            cull.tl[k] = cam->top_left[ax[k]]; cull.right[k] = cam->right[ax[k]]; cull.up[k] = cam->up[ax[k]];
            for (float v : {cam->top_left[ax[k]], cam->right[ax[k]], cam->up[ax[k]]}) {
                uint32_t b;
                std::memcpy(&b, &v, 4);
                key.push_back(b);
            }
        }
        for (float v : {p->real_screen_width, p->real_screen_height}) {
            uint32_t b;
            std::memcpy(&b, &v, 4);
            key.push_back(b);
        }
        key.push_back(c->sat_gen);
    }
    if (c->frame_lists.size() >= kMaxStreamCaches && !c->frame_lists.count(c->stream)) retire_stream_caches(c, nullptr);
    vr_ctx::FrameList& fl = c->frame_lists[c->stream];
    if (key != fl.key) {
        int n_slots = 0, n_total = 0;
        worklist_size(ntx, nty, tx0, tx1, ty0, ty1, &n_slots, &n_total, deal);
        const size_t need = (size_t)std::max(1, n_total) * sizeof(WorkTile);
        if (need > fl.wc.work.bytes) {   // growing frees the old list: the launches reading it first
            ctx_sync(c, c->stream);
            fl.wc.work.ensure(need + 64 * sizeof(WorkTile));
        }
        hip_check(launch_worklist(ntx, nty, tx0, tx1, ty0, ty1, n_slots, fl.wc.work.as<WorkTile>(), cull, deal, c->stream));
        fl.wc.n_work = fl.wc.n_blocks = n_total;
        fl.wc.bg_first = n_slots;
        fl.key = std::move(key);
    }
    return &fl.wc;
}

int project_box_test(const vr_ctx* c, const vr_params* p, const vr_camera* cam, double xy[8][2]);
int hull_edges(const vr_ctx* c, const vr_params* p, const vr_camera* cam, float h[kMaxHull][3]);

// The 8 corners of the dataset box (tightened to the occupied macro cells: a ray outside both meets
// only TF(0) or empty cells, every sample alpha 0) projected onto the screen in pixel units, in
// double precision (orthographic: along front; conic: through the camera position).  Returns 0 when
// nothing can be visible, 2 when no claim can be made (TEST mode, opaque TF(0), a corner behind a
// conic camera, a NaN camera), 1 with the points in xy.
int project_box(const vr_ctx* c, const vr_params* p, const vr_camera* cam, double xy[8][2]) {
    if (p->mode == VR_MODE_TEST) return project_box_test(c, p, cam, xy);
    if (p->mode != VR_MODE_VRC || !c->zero_transparent) return 2;
    double lo[3], hi[3];
    for (int a = 0; a < 3; ++a) {
        if (c->oct.leaf_hi[a] < 0 || c->occ_hi[a] < 0) return 0;   // nothing can be visible
        lo[a] = std::max((double)c->oct.leaf_lo[a], (double)(c->occ_lo[a] << c->cb_shift)) / c->oct.nleaf - 0.5;
        hi[a] = std::min((double)(c->oct.leaf_hi[a] + 1), (double)((c->occ_hi[a] + 1) << c->cb_shift)) / c->oct.nleaf -
                0.5;
    }
    const bool conic = (p->flags & VR_FLAG_CONIC) != 0;
    const double sx = p->width / (double)p->real_screen_width, sy = p->height / (double)p->real_screen_height;
    for (int k = 0; k < 8; ++k) {
        double v[3];
        for (int a = 0; a < 3; ++a) v[a] = ((k >> a) & 1) ? hi[a] : lo[a];
        if (conic) {   // the screen point on the ray pos -> v: where it crosses the plane through tlc
            double n = 0, num = 0;
            for (int a = 0; a < 3; ++a) {
                n += (v[a] - cam->pos[a]) * cam->front[a];
                num += (cam->top_left[a] - cam->pos[a]) * cam->front[a];
            }
            if (n <= 1e-9) return 2;
            const double s = num / n;
            for (int a = 0; a < 3; ++a) v[a] = cam->pos[a] + s * (v[a] - cam->pos[a]);
        }
        double u = 0, w = 0;
        for (int a = 0; a < 3; ++a) {
            u += (v[a] - cam->top_left[a]) * cam->right[a];
            w += (v[a] - cam->top_left[a]) * -cam->up[a];
        }
        xy[k][0] = u * sx;
        xy[k][1] = w * sy;
        if (!std::isfinite(xy[k][0]) || !std::isfinite(xy[k][1])) return 2;
    }
    return 1;
}

// TEST frames (getColorFromNF, kernel.cu:92-115): sample s of pixel (x, y) is p = M (x, y, s, 1) with
// M = toVolume * inverse(lookAt) * modelCam, and a sample outside 0 <= p < d is TF(0) -- with TF(0)
// transparent an exact no-op of either blend.  So a ray whose line misses the dataset box [0, d]^3
// is exactly the background: the box's 8 corners mapped back to (x, y) through M^-1 (double
// precision; the float matrices' rounding is far inside the 2-pixel margin visible_rect adds).
int project_box_test(const vr_ctx* c, const vr_params* p, const vr_camera* cam, double xy[8][2]) {
    if (!c->zero_transparent) return 2;
    CameraState cs;
    cs.pos = {cam->pos[0], cam->pos[1], cam->pos[2]};
    cs.up = {cam->up[0], cam->up[1], cam->up[2]};
    glmf::mat4 mc, iv, tv;
    test_matrices(c->d[0], c->d[1], c->d[2], p->width, p->height, p->samples_per_ray, p->real_screen_width,
                  p->real_screen_height, p->viewplane_distance, cs, &mc, &iv, &tv);
    double A[16], B[16], Cm[16], T1[16], M[16];   // column-major: m[col * 4 + row]
    const float* fm[3] = {reinterpret_cast<const float*>(&mc), reinterpret_cast<const float*>(&iv),
                          reinterpret_cast<const float*>(&tv)};
    for (int i = 0; i < 16; ++i) { A[i] = fm[0][i]; B[i] = fm[1][i]; Cm[i] = fm[2][i]; }
    auto mul = [](const double* X, const double* Y, double* Z) {   // Z = X * Y
        for (int col = 0; col < 4; ++col)
            for (int row = 0; row < 4; ++row) {
                double v = 0;
                for (int k = 0; k < 4; ++k) v += X[k * 4 + row] * Y[col * 4 + k];
                Z[col * 4 + row] = v;
            }
    };
    mul(B, A, T1);
    mul(Cm, T1, M);
    // p = L (x, y, s) + t: invert the 3 x 3 linear part
    const double L[3][3] = {{M[0], M[4], M[8]}, {M[1], M[5], M[9]}, {M[2], M[6], M[10]}};
    const double det = L[0][0] * (L[1][1] * L[2][2] - L[1][2] * L[2][1]) - L[0][1] * (L[1][0] * L[2][2] - L[1][2] * L[2][0]) +
                       L[0][2] * (L[1][0] * L[2][1] - L[1][1] * L[2][0]);
    if (!std::isfinite(det) || std::fabs(det) < 1e-30) return 2;
    double Li[3][3];
    Li[0][0] = (L[1][1] * L[2][2] - L[1][2] * L[2][1]) / det;
    Li[0][1] = (L[0][2] * L[2][1] - L[0][1] * L[2][2]) / det;
    Li[0][2] = (L[0][1] * L[1][2] - L[0][2] * L[1][1]) / det;
    Li[1][0] = (L[1][2] * L[2][0] - L[1][0] * L[2][2]) / det;
    Li[1][1] = (L[0][0] * L[2][2] - L[0][2] * L[2][0]) / det;
    Li[1][2] = (L[0][2] * L[1][0] - L[0][0] * L[1][2]) / det;
    const double t[3] = {M[12], M[13], M[14]};
    for (int k = 0; k < 8; ++k) {
        double v[3];
        for (int a = 0; a < 3; ++a) v[a] = (((k >> a) & 1) ? (double)c->d[a] : 0.0) - t[a];
        for (int r = 0; r < 2; ++r) xy[k][r] = Li[r][0] * v[0] + Li[r][1] * v[1] + Li[r][2] * v[2];
        if (!std::isfinite(xy[k][0]) || !std::isfinite(xy[k][1])) return 2;
    }
    return 1;
}

// Conservative screen-space culling: the rectangle of tiles of a tw x th grid (x-major ids
// t = tx*nty + ty) whose rays can meet the dataset box.  Every other ray samples only TF(0), so
// with TF(0).a == 0 its pixel is exactly the background in either compositing order.  The bounding
// rectangle of the projected box corners is widened by 2 pixels.  Anything project_box makes no
// claim for keeps every tile (all = true).
TileRect visible_rect(const vr_ctx* c, const vr_params* p, const vr_camera* cam, int tw, int th) {
    const int W = p->width, H = p->height;
    const int ntx = (W + tw - 1) / tw, nty = (H + th - 1) / th;
    TileRect all;
    all.tx1 = ntx - 1; all.ty1 = nty - 1;
    TileRect none;
    none.all = false;
    double xy[8][2];
    const int pr = project_box(c, p, cam, xy);
    if (pr == 2) return all;
    if (pr == 0) return none;
    double xmin = 1e300, xmax = -1e300, ymin = 1e300, ymax = -1e300;
    for (int k = 0; k < 8; ++k) {
        xmin = std::min(xmin, xy[k][0]); xmax = std::max(xmax, xy[k][0]);
        ymin = std::min(ymin, xy[k][1]); ymax = std::max(ymax, xy[k][1]);
    }
    const double m = 2.0;
    const double x0 = std::floor(xmin - m), x1 = std::ceil(xmax + m), y0 = std::floor(ymin - m), y1 = std::ceil(ymax + m);
    if (x1 < 0 || y1 < 0 || x0 > W - 1 || y0 > H - 1) return none;
    TileRect r;
    r.all = false;
    r.tx0 = (int)std::max(0.0, std::floor(x0 / tw));
    r.tx1 = (int)std::min((double)ntx - 1, std::floor(x1 / tw));
    r.ty0 = (int)std::max(0.0, std::floor(y0 / th));
    r.ty1 = (int)std::min((double)nty - 1, std::floor(y1 / th));
    if (r.tx0 == 0 && r.ty0 == 0 && r.tx1 == ntx - 1 && r.ty1 == nty - 1) r.all = true;
    return r;
}

// The projected box's convex hull as half-planes in pixel units, for the march's per-workgroup cull
// of the work tiles inside the visible rectangle but off the hull (general views: the projection of
// a rotated box is a hexagon, up to a third of its bounding rectangle).  Edge e keeps the pixels with
// h[e][0] x + h[e][1] y <= h[e][2]; the normals are unit and the offsets widened by the rectangle's
// 2-pixel margin, so every pixel the rectangle test would keep for that reason is kept.  Returns the
// number of edges, 0 = no claim (fewer than 3 hull vertices, or project_box made none).
int hull_edges(const vr_ctx* c, const vr_params* p, const vr_camera* cam, float h[kMaxHull][3]) {
    double xy[8][2];
    if (project_box(c, p, cam, xy) != 1) return 0;
    // Andrew's monotone chain, counter-clockwise in (x, y)
    int idx[8];
    for (int k = 0; k < 8; ++k) idx[k] = k;
    std::sort(idx, idx + 8, [&](int a, int b) {
        return xy[a][0] < xy[b][0] || (xy[a][0] == xy[b][0] && xy[a][1] < xy[b][1]);
    });
    auto cross = [&](int o, int a, int b) {
        return (xy[a][0] - xy[o][0]) * (xy[b][1] - xy[o][1]) - (xy[a][1] - xy[o][1]) * (xy[b][0] - xy[o][0]);
    };
    int hv[16], n = 0;
    for (int i = 0; i < 8; ++i) {
        while (n >= 2 && cross(hv[n - 2], hv[n - 1], idx[i]) <= 0) --n;
        hv[n++] = idx[i];
    }
    for (int i = 6, lower = n + 1; i >= 0; --i) {
        while (n >= lower && cross(hv[n - 2], hv[n - 1], idx[i]) <= 0) --n;
        hv[n++] = idx[i];
    }
    --n;   // the last point repeats the first
    if (n < 3 || n > kMaxHull) return 0;
    double area = 0;
    for (int i = 0; i < n; ++i) area += cross(hv[0], hv[i], hv[(i + 1) % n]);
    if (!(area > 1.0)) return 0;   // degenerate (a segment or a sliver of a pixel): no claim
    const double m = 2.0;
    for (int i = 0; i < n; ++i) {
        const double* a = xy[hv[i]];
        const double* b = xy[hv[(i + 1) % n]];
        // counter-clockwise: the outward normal of edge a -> b is (dy, -dx)
        double nx = b[1] - a[1], ny = -(b[0] - a[0]);
        const double len = std::sqrt(nx * nx + ny * ny);
        if (!(len > 0)) return 0;
        nx /= len; ny /= len;
        // float rounding of the stored edge: one more pixel of margin covers it with room to spare
        h[i][0] = (float)nx;
        h[i][1] = (float)ny;
        h[i][2] = (float)(nx * a[0] + ny * a[1] + m + 1.0);
    }
    return n;
}

std::vector<int32_t> visible_tiles_uncached(const vr_ctx* c, const vr_params* p, const vr_camera* cam, int tw, int th);

// The view axis of an axis-parallel orthographic VRC view whose empty cell columns may be culled
// (cull >= 2, TF(0) transparent, a finite camera with exactly one non-zero front component), else -1.
// Along such a view a ray's other two coordinates are constant, so a ray whose cell column holds no
// occupied cell samples only alpha-0 classes and TF(0): exactly the background.
int cull_axis(const vr_ctx* c, const vr_params* p, const vr_camera* cam) {
    if (!(c->cull >= 2 && p->mode == VR_MODE_VRC && c->zero_transparent && !(p->flags & VR_FLAG_CONIC) &&
          c->col_sat[0].size() == (size_t)(c->ncell + 1) * (c->ncell + 1)))
        return -1;
    int nz = 0, ma = -1;
    for (int a = 0; a < 3; ++a)
        if (cam->front[a] != 0.0f) { ++nz; ma = a; }
    bool finite = true;
    for (int a = 0; a < 3; ++a)
        finite = finite && std::isfinite(cam->top_left[a]) && std::isfinite(cam->right[a]) && std::isfinite(cam->up[a]);
    return nz == 1 && finite ? ma : -1;
}

std::vector<int32_t> visible_tiles(const vr_ctx* c, const vr_params* p, const vr_camera* cam, int tw, int th) {
    std::vector<uint32_t> key(sizeof(vr_params) / 4 + sizeof(vr_camera) / 4 + 3);
    std::memcpy(key.data(), p, sizeof(vr_params));
    std::memcpy(key.data() + sizeof(vr_params) / 4, cam, sizeof(vr_camera));
    key[key.size() - 3] = (uint32_t)tw; key[key.size() - 2] = (uint32_t)th; key[key.size() - 1] = (uint32_t)c->cull;
    auto it = c->vis_cache.find(key);
    if (it != c->vis_cache.end()) return it->second;
    std::vector<int32_t> v = visible_tiles_uncached(c, p, cam, tw, th);
    if (c->vis_cache.size() >= 256) c->vis_cache.clear();
    c->vis_cache.emplace(std::move(key), v);
    return v;
}

std::vector<int32_t> visible_tiles_uncached(const vr_ctx* c, const vr_params* p, const vr_camera* cam, int tw, int th) {
    const int nty = (p->height + th - 1) / th;
    const TileRect r = visible_rect(c, p, cam, tw, th);
    // (cull >= 2) the rectangle's tiles separated from the projected box's hull by one of its edges
    // are dropped too: the same test as the march's workgroup cull, on the tile's pixel range
    float h[kMaxHull][3];
    const int nh = c->cull >= 2 ? hull_edges(c, p, cam, h) : 0;
    // (cull >= 2) axis-parallel orthographic views (front along volume axis ma, rays parallel to it):
    // a ray's other two coordinates are constant, so a ray whose cell column along ma holds no
    // occupied cell samples only alpha-0 classes and TF(0) -- exactly the background -- and so is
    // a tile all of whose rays' columns are empty.  The columns a tile's rays can reach: the ray
    // origins' q range over the tile's corner pixels (q is affine in the pixel), one leaf of margin.
    const int ma = cull_axis(c, p, cam);
    auto columns_empty = [&](int px0, int px1, int py0, int py1) {
        const int a0 = ma == 0 ? 1 : 0, a1 = ma == 2 ? 1 : 2;
        const double L = (double)c->oct.nleaf;
        int lo[2], hi[2];
        const int ax[2] = {a0, a1};
        for (int k = 0; k < 2; ++k) {
            const int a = ax[k];
            double qmin = 1e300, qmax = -1e300;
            for (int cx = 0; cx < 2; ++cx)
                for (int cy = 0; cy < 2; ++cy) {
                    const double x = cx ? px1 : px0, y = cy ? py1 : py0;
                    const double q = (double)cam->top_left[a] + (x * p->real_screen_width / p->width) * cam->right[a] +
                                     (y * p->real_screen_height / p->height) * -(double)cam->up[a] + 0.5;
                    qmin = std::min(qmin, q); qmax = std::max(qmax, q);
                }
            const double l0 = std::floor(qmin * L) - 1.0, l1 = std::floor(qmax * L) + 1.0;
            if (l1 < 0.0 || l0 > L - 1.0) return true;   // outside the cube on this axis: TF(0) only
            lo[k] = (int)std::max(0.0, l0) >> c->cb_shift;
            hi[k] = (int)std::min(L - 1.0, l1) >> c->cb_shift;
        }
        const std::vector<int32_t>& S = c->col_sat[ma];
        const size_t side = (size_t)c->ncell + 1;
        const int32_t n = S[(size_t)(hi[0] + 1) * side + (size_t)(hi[1] + 1)] - S[(size_t)lo[0] * side + (size_t)(hi[1] + 1)] -
                          S[(size_t)(hi[0] + 1) * side + (size_t)lo[1]] + S[(size_t)lo[0] * side + (size_t)lo[1]];
        return n == 0;
    };
    // (cull >= 2) other orthographic views: the tiles the occupied super cells' projections can
    // reach (each super cell's projected bounding rectangle, widened by 2 pixels like the box's): a
    // ray off all of them meets only empty cells and TF(0) -- exactly the background
    std::vector<uint8_t> mark;
    if (c->cull >= 2 && ma < 0 && nh > 0 && p->mode == VR_MODE_VRC && !(p->flags & VR_FLAG_CONIC) &&
        !c->socc.empty()) {
        const int ntx = (p->width + tw - 1) / tw;
        mark.assign((size_t)ntx * nty, 0);
        const double sxs = p->width / (double)p->real_screen_width, sys = p->height / (double)p->real_screen_height;
        const double L = (double)c->oct.nleaf, SL = (double)(1 << (c->cb_shift + c->sc_shift));
        double er = 0, eu = 0;   // screen half-extent of a super cell (per unit half-edge)
        for (int a = 0; a < 3; ++a) { er += std::fabs((double)cam->right[a]); eu += std::fabs((double)cam->up[a]); }
        for (int i = 0; i < c->nsc; ++i)
            for (int j = 0; j < c->nsc; ++j)
                for (int k = 0; k < c->nsc; ++k) {
                    if (!c->socc[((size_t)i * c->nsc + j) * c->nsc + k]) continue;
                    const int ci[3] = {i, j, k};
                    double u = 0, w = 0, half = 0;
                    for (int a = 0; a < 3; ++a) {
                        const double l0 = ci[a] * SL, l1 = std::min(L, (ci[a] + 1) * SL);
                        const double ctr = 0.5 * (l0 + l1) / L - 0.5;   // world coordinate (q - 0.5)
                        half = std::max(half, 0.5 * (l1 - l0) / L);
                        u += (ctr - cam->top_left[a]) * cam->right[a];
                        w += (ctr - cam->top_left[a]) * -(double)cam->up[a];
                    }
                    const double m = 2.0;
                    const double x0 = (u - half * er) * sxs - m, x1 = (u + half * er) * sxs + m;
                    const double y0 = (w - half * eu) * sys - m, y1 = (w + half * eu) * sys + m;
                    const int tx0 = (int)std::max(0.0, std::floor(x0 / tw)), tx1 = (int)std::min(ntx - 1.0, std::floor(x1 / tw));
                    const int ty0 = (int)std::max(0.0, std::floor(y0 / th)), ty1 = (int)std::min(nty - 1.0, std::floor(y1 / th));
                    for (int tx = tx0; tx <= tx1; ++tx)
                        for (int ty = ty0; ty <= ty1; ++ty) mark[(size_t)tx * nty + ty] = 1;
                }
    }
    std::vector<int32_t> keep;
    for (int tx = r.tx0; tx <= r.tx1; ++tx)
        for (int ty = r.ty0; ty <= r.ty1; ++ty) {
            bool off = false;
            for (int e = 0; e < nh && !off; ++e) {
                const double px = h[e][0] > 0.0f ? tx * tw : std::min(p->width, (tx + 1) * tw) - 1;
                const double py = h[e][1] > 0.0f ? ty * th : std::min(p->height, (ty + 1) * th) - 1;
                off = (double)h[e][0] * px + (double)h[e][1] * py > (double)h[e][2];
            }
            if (!off && ma >= 0)
                off = columns_empty(tx * tw, std::min(p->width, (tx + 1) * tw) - 1, ty * th,
                                    std::min(p->height, (ty + 1) * th) - 1);
            if (!off && !mark.empty()) off = !mark[(size_t)tx * nty + ty];
            if (!off) keep.push_back(tx * nty + ty);
        }
    return keep;
}

void check_params(const vr_params* p) {
    if (!p || p->width <= 0 || p->height <= 0 || p->samples_per_ray <= 0 || p->width > 65535 || p->height > 65535)
        throw Error(VR_EINVAL, "vr_params: bad width/height/samples_per_ray");
    if (p->mode != VR_MODE_VRC && p->mode != VR_MODE_TEST) throw Error(VR_EINVAL, "vr_params: unknown mode");
    if (p->flags & ~(VR_FLAG_ESS | VR_FLAG_ERT | VR_FLAG_SHADE | VR_FLAG_CONIC))
        throw Error(VR_EINVAL, "vr_params: unknown flags");
    if ((p->flags & (VR_FLAG_SHADE | VR_FLAG_CONIC)) && p->mode != VR_MODE_VRC)
        throw Error(VR_EINVAL, "vr_params: VR_FLAG_SHADE / VR_FLAG_CONIC are defined for VR_MODE_VRC only");
}

VrcFrame make_vrc(const vr_ctx* c, const vr_params* p, const vr_camera* cam) {
    VrcFrame f;
    std::memset(&f, 0, sizeof f);
    f.W = p->width; f.H = p->height; f.S = p->samples_per_ray; f.flags = p->flags;
    f.rsw = p->real_screen_width; f.rsh = p->real_screen_height;
    f.sd = p->sample_distance; f.fc = p->front_clip_plane;
    for (int i = 0; i < 3; ++i) {
        f.tlc[i] = cam->top_left[i]; f.right[i] = cam->right[i]; f.up[i] = cam->up[i]; f.front[i] = cam->front[i];
    }
    for (int i = 0; i < 4; ++i) f.bg[i] = p->background[i];
    f.ert_eps = (p->flags & VR_FLAG_ERT) ? p->ert_epsilon : 0.0f;
    f.d2d3 = c->d[1] * c->d[2]; f.d3 = c->d[2];
    f.depth = (int)c->oct.maximum_depth;
    f.nleaf = c->oct.nleaf;
    f.leaves = (float)c->oct.nleaf;
    f.cb_shift = c->cb_shift;
    f.ncell = c->ncell;
    f.cell_q = (float)(1 << c->cb_shift) / (float)c->oct.nleaf;
    f.shrink_q = 0.05f / (float)c->oct.nleaf;   // ESS margin: 0.05 leaf >> float position error
    for (int a = 0; a < 3; ++a) {
        f.step[a] = f.sd * f.front[a];
        f.inv_step[a] = f.step[a] != 0.0f ? 1.0f / f.step[a] : 0.0f;
    }
    f.occ_words = (int)(((int64_t)c->ncell * c->ncell * c->ncell + 31) / 32);
    f.occ_lds = (f.occ_words <= 8192 && c->occ_lds) ? 1 : 0;
    {   // orthographic view along a volume axis: exactly one non-zero component of front
        int nz = 0, ax = -1;
        for (int a = 0; a < 3; ++a)
            if (f.front[a] != 0.0f) { ++nz; ax = a; }
        // the march then tabulates q(s) along the axis once per frame: that needs the march-axis
        // coordinate to be ray-independent (right, up without a component there), finite camera
        // values (q monotone in s) and a table that fits LDS
        bool finite = std::isfinite(f.sd) && std::isfinite(f.fc);
        for (int a = 0; a < 3; ++a)
            finite = finite && std::isfinite(f.tlc[a]) && std::isfinite(f.right[a]) && std::isfinite(f.up[a]) &&
                     std::isfinite(f.front[a]);
        // (the march-axis map is staged as int32: not the 64-bit x map of IDX64 volumes)
        const bool tab_ok = ax >= 0 && f.right[ax] == 0.0f && f.up[ax] == 0.0f && finite && f.S <= kMaxTabSamples &&
                            !(c->idx64 && ax == 0);
        f.axis1 = (nz == 1 && tab_ok && c->axis1_ok && !(p->flags & VR_FLAG_CONIC)) ? ax : -1;
    }
    for (int a = 0; a < 3; ++a) {
        const float margin = 1e-5f;
        if (c->oct.leaf_hi[a] < 0) { f.box_lo[a] = 2.0f; f.box_hi[a] = -2.0f; continue; }
        f.box_lo[a] = (float)c->oct.leaf_lo[a] / (float)c->oct.nleaf - margin;
        f.box_hi[a] = (float)(c->oct.leaf_hi[a] + 1) / (float)c->oct.nleaf + margin;
    }
    f.conic = (p->flags & VR_FLAG_CONIC) ? 1 : 0;
    for (int a = 0; a < 3; ++a) f.campos[a] = cam->pos[a];
    f.zero_transparent = c->zero_transparent ? 1 : 0;
    // can a marched sample lie outside the unit cube?  Without clipping, yes; with it, only if the
    // clip margin (<= 3 samples) around the dataset box crosses a cube face.
    f.edge_guard = (f.zero_transparent && !f.conic) ? 0 : 1;
    for (int a = 0; a < 3; ++a) {
        const float m = 4.0f * std::fabs(f.step[a]) + 1e-4f;
        if (f.box_lo[a] <= f.box_hi[a] && (f.box_lo[a] < m || f.box_hi[a] > 1.0f - m)) f.edge_guard = 1;
    }
    f.cls0 = c->cls0_vrc;
    // general orthographic views with the clip active: LDS leaf maps padded with kMapOut so the
    // march's batches index them without clamps (vr_kernels.hip).  Every sample a batch evaluates
    // lies within (K + 3) steps of the dataset box (clip margins -1 / +2 samples, batches of K <= 16
    // past s_end), i.e. within (K + 3) |step_c| 2^D leaves of it per axis; the pad covers that with
    // room to spare, and is off when it would exceed 64 leaves (very long steps).
    f.pad = 0;
    f.leafcols = c->leafcols ? 1 : 0;
    if (c->opt.leaf_map_pad && f.axis1 < 0 && !f.conic && f.zero_transparent && !c->idx64 && f.S <= kMaxTabSamples) {
        bool finite = std::isfinite(f.sd) && std::isfinite(f.fc);
        float mstep = 0.0f;
        for (int a = 0; a < 3; ++a) {
            finite = finite && std::isfinite(f.tlc[a]) && std::isfinite(f.right[a]) && std::isfinite(f.up[a]) &&
                     std::isfinite(f.front[a]) && std::isfinite(f.step[a]);
            mstep = std::max(mstep, std::fabs(f.step[a]));
        }
        const double P = std::ceil((16.0 + 6.0) * (double)mstep * (double)f.nleaf) + 4.0;
        // (a multiple of 4: the march stages the padded maps in whole int4s)
        if (finite && P <= 64.0) f.pad = ((int32_t)P + 3) & ~3;
    }
    f.ka = p->shade_ambient; f.kd = p->shade_diffuse; f.ks = p->shade_specular; f.shininess = p->shade_shininess;
    f.d1i = (int)c->d[0]; f.d2i = (int)c->d[1]; f.d3i = (int)c->d[2];
    f.bg_first = INT32_MAX;   // no background-only workgroups unless launch_frame sets them
    f.bg_group = 1;
    // general views (axis-aligned ones project the box to its own bounding rectangle): the hull of
    // the projected box, for the march's workgroup cull of the rectangle's corners
    f.n_hull = (c->cull >= 2 && f.axis1 < 0) ? hull_edges(c, p, cam, f.hull) : 0;
    return f;
}

// TEST axis views (test_axis_kernel): the march axis's per-frame tables as the kernel lays them out in
// LDS from s_ztab on -- per sample int2 {(int)p_a | delta << 29 (-1 outside [0, d_a)), bits of
// p_a - (int)p_a}, then (ESS) per sample the int8 cell of (int)p_a (-1 below, tnca at or past the
// top) padded to 4 B, then per cell the first sample in march order whose cell is it or beyond it in
// the direction of travel (F2B: S if none; B2F: -1 if none).  The kernel's own expressions in IEEE
// float (no contraction on either side), so the same table bit for bit; every workgroup then stages
// it in 16-B loads instead of building it (round 5).  Returns the table's int32 words.
int make_test_axis_table(const TestFrame& f, bool f2b, bool ess, std::vector<int32_t>& out) {
    const int ax = f.axt, S = f.S;
    const float fda = ax == 0 ? f.fd1 : (ax == 1 ? f.fd2 : f.fd3);
    const int tca = f.tca[ax], tnca = f.tnca[ax];
    const bool cells_up = f2b ? f.axt_up != 0 : f.axt_up == 0;   // the kernel's UP
    const int words = 2 * S + (ess ? (S + 3) / 4 + tnca : 0);
    // (32 words of slack: the kernel's staging reads 16 B past the end, its scalar loads of a batch's
    // K <= 16 entries up to 120 B past the last one)
    out.assign((size_t)words + 32, 0);
    std::vector<int> cel(ess ? (size_t)S : 0);
    for (int s = 0; s < S; ++s) {
        const float q1z = f.mc[10] * (float)s + f.mc[14];
        const float q2 = 0.0f + (f.iv[8 + ax] * q1z + f.iv[12 + ax] * 1.0f);
        const float pa = f.tv[5 * ax] * q2 + f.tv[12 + ax];
        const int i0 = (int)pa, i1 = (int)(pa + 1.0f);
        const bool in = pa >= 0.0f && pa < fda;
        const float fr = pa - (float)(int)pa;
        int32_t fb;
        std::memcpy(&fb, &fr, 4);
        out[(size_t)2 * s] = in ? (i0 | ((i1 - i0) << 29)) : -1;
        out[(size_t)2 * s + 1] = fb;
        if (ess) cel[(size_t)s] = in ? i0 / tca : (pa < 0.0f ? -1 : tnca);
    }
    if (ess) {
        int8_t* zc = reinterpret_cast<int8_t*>(out.data() + 2 * S);
        for (int s = 0; s < S; ++s) zc[s] = (int8_t)cel[(size_t)s];
        int32_t* ze = out.data() + 2 * S + (S + 3) / 4;
        for (int c = 0; c < tnca; ++c) {
            auto beyond = [&](int s) { return cells_up ? cel[(size_t)s] >= c : cel[(size_t)s] <= c; };
            int v = f2b ? S : -1;
            if (f2b) {
                for (int s = 0; s < S; ++s) if (beyond(s)) { v = s; break; }
            } else {
                for (int s = S - 1; s >= 0; --s) if (beyond(s)) { v = s; break; }
            }
            ze[c] = v;
        }
    }
    return words;
}

TestFrame make_test(const vr_ctx* c, const vr_params* p, const vr_camera* cam) {
    TestFrame f;
    std::memset(&f, 0, sizeof f);
    f.W = p->width; f.H = p->height; f.S = p->samples_per_ray; f.flags = p->flags;
    CameraState cs;
    cs.pos = {cam->pos[0], cam->pos[1], cam->pos[2]};
    cs.up = {cam->up[0], cam->up[1], cam->up[2]};
    glmf::mat4 mc, iv, tv;
    test_matrices(c->d[0], c->d[1], c->d[2], p->width, p->height, p->samples_per_ray, p->real_screen_width,
                  p->real_screen_height, p->viewplane_distance, cs, &mc, &iv, &tv);
    std::memcpy(f.mc, &mc, 64); std::memcpy(f.iv, &iv, 64); std::memcpy(f.tv, &tv, 64);
    {   // modelCam and toVolume separable (zero off-diagonal products, finite entries): the march
        // then skips their zero terms, bit for bit (test_march_kernel, SEP)
        bool sep = true;
        for (int i : {1, 2, 4, 6, 8, 9}) sep = sep && f.mc[i] == 0.0f && f.tv[i] == 0.0f;
        for (int i : {0, 5, 10, 12, 13, 14}) sep = sep && std::isfinite(f.mc[i]) && std::isfinite(f.tv[i]);
        for (int i = 0; i < 16; ++i) sep = sep && std::isfinite(f.iv[i]);
        f.sep = sep ? 1 : 0;
        // the general march's per-frame table of the ray-independent half of the position: 16 B per
        // sample of [-4, S + 4) in LDS, bounded (unbounded it failed the launch from
        // S ~ 9k); longer rays compute it per sample with the same expressions
        f.sep_tab = (sep && (int64_t)f.S + 8 <= kMaxTestTab) ? 1 : 0;
    }
    for (int i = 0; i < 4; ++i) f.bg[i] = p->background[i];
    f.ert_eps = (p->flags & VR_FLAG_ERT) ? p->ert_epsilon : 0.0f;
    f.d1 = c->d[0]; f.d2 = c->d[1]; f.d3 = c->d[2];
    f.total = c->d[0] * c->d[1] * c->d[2];
    f.fd1 = (float)c->d[0]; f.fd2 = (float)c->d[1]; f.fd3 = (float)c->d[2];
    f.zero_transparent = c->zero_transparent ? 1 : 0;
    f.cls0 = c->cls0_test;
    f.idx64 = (f.total + f.d2 * f.d3 + f.d3 + 1) >= ((int64_t)1 << 31) ? 1 : 0;
    f.tcb = c->tcb;
    for (int a = 0; a < 3; ++a) f.tnc[a] = c->tnc[a];
    f.occ_words = (int)(((int64_t)c->tnc[0] * c->tnc[1] * c->tnc[2] + 31) / 32);
    f.occ_lds = (f.occ_words <= 8192 && c->occ_lds) ? 1 : 0;
    {   // axis views (test_axis_kernel) along a, fixed axes b, c: iv[8+b] = iv[8+c] = 0 make
        // iv[8+r] q1z a signed zero u, and u + iv[12+r] = iv[12+r] exactly unless iv[12+r] is -0; then
        // A_r + (u + iv[12+r]) is A_r itself for A_r != 0, and a signed zero otherwise, which
        // tv_rr (+-0) + tv[12+r] maps to tv[12+r] whenever tv[12+r] != 0 (it is d_r / 2): p_b, p_c
        // fixed per ray, bit for bit.  The plane march also needs 32-bit corner indices, class
        // 0 = TF(0) (the buffer bound is the reference's idx < total guard) and TF(0) transparent
        // (alpha-0 samples skipped).
        auto negzero = [](float v) { return v == 0.0f && std::signbit(v); };
        // The per-frame table along a also needs iv[a] = iv[4+a] = 0 (A_a a signed zero) and
        // tv[12+a] != 0, and S <= 4096 (8 B per sample of LDS), d_a < 2^28 (packed corner index: the
        // voxel i0 < d_a sits below the 2-bit delta at bit 29; 2^29 would be exact too, 2^28 keeps
        // one bit of margin).  Along x and y the two z corners of a line pair are read as one dword.
        f.axt = -1;
        const bool common = f.sep && f.S <= 4096 && !f.idx64 && f.cls0 == 0 && f.zero_transparent && c->test_axz;
        for (int a = 2; a >= 0 && common && f.axt < 0; --a) {
            const int b = a == 0 ? 1 : 0, cc = a == 2 ? 1 : 2;
            auto fixed = [&](int r) { return f.iv[8 + r] == 0.0f && (!negzero(f.iv[12 + r]) || f.tv[12 + r] != 0.0f); };
            if (fixed(b) && fixed(cc) &&
                f.iv[a] == 0.0f && f.iv[4 + a] == 0.0f && f.tv[12 + a] != 0.0f && c->d[a] < (1 << 28))
                f.axt = a;
        }
        f.axt_up = f.axt >= 0 && (double)f.tv[5 * f.axt] * (double)f.iv[8 + f.axt] * (double)f.mc[10] > 0.0 ? 1 : 0;
        if (f.axt >= 0) {
            // the march axis's clip range, once per frame: test_axis_kernel's p_a(s) with A_a = +-0
            // (A_a + u = u for u != 0; u = +-0 gives tv[12+a] either way, tv[12+a] != 0 above), the
            // same float and double operations as its per-ray statement (IEEE on host and device, no
            // contraction), so the same [s_begin, s_end) bit for bit
            const int a = f.axt;
            auto pa_of = [&](int s) -> float {
                const float q1z = f.mc[10] * (float)s + f.mc[14];
                const float q2 = 0.0f + (f.iv[8 + a] * q1z + f.iv[12 + a] * 1.0f);
                return f.tv[5 * a] * q2 + f.tv[12 + a];
            };
            const double b0 = pa_of(0), b1 = pa_of(f.S > 1 ? f.S - 1 : 0);
            const double st = f.S > 1 ? (b1 - b0) / (double)(f.S - 1) : 0.0;
            const double base[3] = {b0, b0, b0}, stp[3] = {st, st, st};
            const float fd = a == 0 ? f.fd1 : (a == 1 ? f.fd2 : f.fd3);
            const float lo[3] = {-0.01f, -0.01f, -0.01f}, hi[3] = {fd + 0.01f, fd + 0.01f, fd + 0.01f};
            // (one axis: the three entries are the same constraint)
            clip_range(base, stp, lo, hi, f.S, f.ax_sb, f.ax_se);
        }
    }
    // whole frames of general views: the hull of the dataset box's projection (project_box_test);
    // work tiles off it are the background (test_background in vr_test.hip)
    f.n_hull = (c->cull >= 2 && f.axt < 0) ? hull_edges(c, p, cam, f.hull) : 0;
    f.cv = c->tcc.p != nullptr ? c->tcv : 0;
    f.cv_bytes = (int32_t)c->tcv_bytes;
    f.mul24 = (c->d[0] < (1 << 24) && c->d[1] * c->d[2] < (1 << 24)) ? 1 : 0;
    f.lin = c->test_faces_dirty == 0 ? 1 : 0;   // (classify: test_faces_kernel)
    for (int a = 0; a < 3; ++a) {   // (test_march_kernel's corner-volume test; dims < 2^24, so d + 1 is exact)
        const float top = (float)(c->d[a] + 1);
        const float ulp = std::nextafter(top, std::numeric_limits<float>::infinity()) - top;
        f.wthr[a] = 1.0f - ulp;
    }
    for (int a = 0; a < 3; ++a) {
        f.tca[a] = c->tca[a];
        f.tnca[a] = c->tnca[a];
        f.tcol_pitch[a] = c->tcol_pitch[a];
        f.tcol_base[a] = c->tcol_base[a];
    }
    return f;
}

void launch_frame(vr_ctx* c, const vr_params* p, const vr_camera* cam, WorkCache* wc, float4* out, int out_tiles,
                  int tile_w, int tile_h, int out_rgb) {
    WorkView wv;
    wv.work = wc->work.as<WorkTile>();
    wv.n_work = wc->n_work;
    wv.n_blocks = wc->n_blocks;
    wv.bg_first = wc->bg_first;
    launch_frame(c, p, cam, wv, out, out_tiles, tile_w, tile_h, out_rgb);
}

void launch_frame(vr_ctx* c, const vr_params* p, const vr_camera* cam, const WorkView& wv, float4* out, int out_tiles,
                  int tile_w, int tile_h, int out_rgb) {
    const WorkView* wc = &wv;
    if (wc->n_blocks == 0) return;
    std::pair<hipEvent_t, hipEvent_t> ev{nullptr, nullptr};
    if (c->timing) {
        if (c->ev_free.empty()) {
            hip_check(hipEventCreate(&ev.first));
            hip_check(hipEventCreate(&ev.second));
        } else {
            ev = c->ev_free.back();
            c->ev_free.pop_back();
        }
        hip_check(hipEventRecord(ev.first, c->stream));
    }

    if (p->mode == VR_MODE_VRC) {
        if ((p->flags & VR_FLAG_SHADE) && !c->nrm.p) {   // per-voxel normals, built on first shaded frame
            const int64_t n = c->d[0] * c->d[1] * c->d[2];
            c->nrm.ensure((size_t)n * sizeof(float4));
            hip_check(launch_normals(c->vol.as<float>(), c->d[0], c->d[1], c->d[2], c->nrm.as<float4>(), c->stream));
        }
        VrcFrame f = make_vrc(c, p, cam);
        // exact back-to-front frames march with empty-space skipping: skipping an alpha-0 sample is
        // bitwise exact back to front (r * (1 - 0) + c * 0 = r, the reference's blend).  Axis-aligned
        // views: column masks (C3 82 -> 61 us, C5 5.37 -> 2.68 ms); general orthographic views: the
        // lazy cell-distance test (oblique 90 -> 87 us).  Conic views and TEST keep the plain march.
        if (c->opt.exact_skip && !(f.flags & (VR_FLAG_ESS | VR_FLAG_ERT | VR_FLAG_SHADE)) && !f.conic &&
            f.zero_transparent)
            f.flags |= VR_FLAG_ESS;
        f.out_tiles = out_tiles; f.tile_w = tile_w; f.tile_h = tile_h; f.n_work = wc->n_work; f.out_rgb = out_rgb;
        f.n_slots = wc->n_blocks;
        f.persist_wgs = c->persist_wgs;
        // whole frames: the culled (background-only) work tiles are stored kBgGroup per workgroup --
        // fewer workgroups to dispatch for the same 16 B per pixel
        f.bg_first = wc->n_work;
        f.bg_group = 1;
        int n_launch = wc->n_blocks;
        if (!out_tiles && c->persist_wgs == 0 && wc->bg_first > 0 && wc->bg_first < wc->n_work) {
            f.bg_first = wc->bg_first;
            f.bg_group = kBgGroup;
            n_launch = wc->bg_first + (wc->n_work - wc->bg_first + kBgGroup - 1) / kBgGroup;
            f.n_slots = n_launch;
        }
        // the volume this view marches: general views of a compact 32-bit volume take its byte copy
        const bool use_gen = c->gen && f.axis1 < 0;
        const int cb = use_gen ? 8 : c->cbits;
        const int64_t vbytes = use_gen ? c->gen_bytes : c->cls_bytes;
        f.cls_bytes = c->idx64 ? 0 : (int32_t)vbytes;
        // class addressing: bits (o >> 3, bit o & 7) below 8 bits per class, bytes at 8
        f.cbits = cb;
        f.osh = cb < 8 ? 3 : 0;
        f.omask = cb < 8 ? 7 : 0;
        f.mapout_ok = (cb < 8 ? vbytes * 8 : vbytes) < ((int64_t)1 << 29) ? 1 : 0;
        // run words (views along z): 8-byte words of the class volume, whose bytes are a multiple of 8
        // (128-byte default bricks) so every word lies inside it
        f.qsh = cb < 8 ? 6 : 3;
        f.bsh = cb < 8 ? 0 : 3;
        f.zrun = (f.axis1 == 2 && vbytes % 8 == 0 &&
                  (c->opt.run_words == 2 || (c->opt.run_words == 0 && c->idx64))) ? 1 : 0;
        // a batch's K samples advance |step_z| 2^D leaves each: the leaf index moves at most
        // floor((K - 1) |step_z| 2^D + 1) over the batch (a tiny margin for the per-sample roundings),
        // the voxel index as much when L = 2^D (the leaf map is a shift) or one more than the scaled
        // leaf span otherwise; a voxel span of at most bz touches at most two z-bricks.  Two z-bricks
        // are two WORDS only when every z-run lies inside one aligned 8-byte word: runs start at
        // multiples of their length bz * cb bits (bricks are contiguous), so that needs bz * cb to
        // divide 64 (e.g. not bz = 16 at 8 bits, nor bz = 3, 5, 6); otherwise the batch keeps the
        // per-sample miss test
        if (f.zrun) {
            const double dl = std::fabs((double)f.step[2]) * (double)c->oct.nleaf;
            const double leaf_span =
                std::floor((double)(vrc_batch_of(f, c->batch) - 1) * dl * (1.0 + 1e-6) + 1.0 + 1e-4);
            const double L = (double)c->oct.longest_dimension;
            const double vox_span = (L == (double)c->oct.nleaf) ? leaf_span
                                                                : std::floor(leaf_span * L / (double)c->oct.nleaf) + 1.0;
            const int run_bits = c->brick[2] * cb;
            f.zspan2 = (vox_span <= (double)c->brick[2] && run_bits <= 64 && 64 % run_bits == 0) ? 1 : 0;
        }
        f.c0_noop = (!c->tf.empty() && c->tf[0].rgba[3] == 0.0f) ? 1 : 0;
        // split view table (views along z, 32-bit volumes): the rays' (x, y) offsets are whole bytes
        // when a brick's z-run is (build_layout: bz * cbits a multiple of 8)
        f.tsplit = (f.axis1 == 2 && !c->idx64 && !f.zrun && !(f.flags & VR_FLAG_SHADE) && c->opt.table_split &&
                    (cb == 8 || (c->brick[2] * cb) % 8 == 0)) ? 1 : 0;
        const uint8_t* vcls = use_gen ? c->cls_gen.as<uint8_t>() : c->cls_vrc.as<uint8_t>();
        // general 32-bit views stage their LDS maps from the kMapPadMax-padded copy (vrc_march_kernel)
        const bool gen_view = f.axis1 < 0 || f.conic;
        const int32_t* vmaps = (gen_view && !c->idx64)
                                   ? (use_gen ? c->pmaps_gen_pad.as<int32_t>() : c->pmaps_pad.as<int32_t>())
                                   : (use_gen ? c->pmaps_gen.as<int32_t>() : c->pmaps.as<int32_t>());
        // AXIS1 view table (a function of the view alone): the first launch of a view builds it in
        // every workgroup and workgroup 0 publishes a copy; later launches of the same view stage the
        // copy (one round of loads) instead of rebuilding it.  Any change of an input is a new view.
        const int32_t* gtab = nullptr;
        int32_t* gtab_out = nullptr;
        std::vector<uint32_t> pub_key;
        if (c->tab_reuse && f.axis1 >= 0 && !f.conic) {
            const int ma = f.axis1;
            const float kf[] = {f.sd, f.fc, f.tlc[ma], f.right[ma], f.up[ma], f.front[ma], f.step[ma], f.leaves};
            const int ki[] = {ma, f.S, f.flags, f.zero_transparent, c->batch, f.ncell, f.cb_shift, f.tsplit, f.zrun, f.cbits};
            std::vector<uint32_t> key(sizeof kf / 4 + sizeof ki / 4);
            std::memcpy(key.data(), kf, sizeof kf);
            std::memcpy(key.data() + sizeof kf / 4, ki, sizeof ki);
            if (c->axtab.size() >= kMaxStreamCaches && !c->axtab.count(c->stream))   // (tables may be in flight: retired)
                retire_stream_caches(c, nullptr);
            vr_ctx::AxTab& at = c->axtab[c->stream];
            if (key == at.key) {
                gtab = at.buf.as<int32_t>();
            } else {
                at.key.clear();
                const size_t tb = vrc_axis1_table_bytes(f, c->batch);
                if (tb + 16 > at.buf.bytes) ctx_sync(c, c->stream);   // growing frees the old copy
                at.buf.ensure(tb + 16);   // (the march stages it in whole int4s)
                gtab_out = at.buf.as<int32_t>();
                pub_key = std::move(key);
            }
        }
#if VR_DIAG_STATS
        // diagnostic build only (make DIAG=1): per-lane work statistics to stderr, records to VR_STATS_DUMP
        if (!c->idx64) {
            DevBuf sb;
            const size_t nw = (size_t)wc->n_blocks * 4;
            const size_t words = nw * 6 + nw * 64 * 2;
            sb.ensure(words * 8);
            hip_check(hipMemsetAsync(sb.p, 0, words * 8, c->stream));
            VrcFrame fs = f;
            hip_check(launch_vrc_stats(fs, wc->work, nullptr, wc->n_blocks, vcls, vmaps, c->occ.as<uint32_t>(),
                                       c->tf_rgba.as<float4>(), (int)c->tf.size(), out, sb.as<unsigned long long>(),
                                       c->stream, (c->leafcols ? c->occ_leafcols : c->occ_cols).as<unsigned long long>(), c->cdist_p, gtab));
            std::vector<unsigned long long> h(words);
            hip_check(hipMemcpyAsync(h.data(), sb.p, words * 8, hipMemcpyDeviceToHost, c->stream));
            hip_check(hipStreamSynchronize(c->stream));
            unsigned long long lanes = 0, iters = 0, jumps = 0, loads = 0, wmax_inner = 0, wmax_loads = 0, busy = 0;
            for (size_t w = 0; w < nw; ++w) {
                unsigned mi = 0, ml = 0;
                for (int l = 0; l < 64; ++l) {
                    const unsigned long long* r = &h[nw * 6 + 2 * (w * 64 + l)];
                    if (!(r[1] >> 63)) continue;
                    const unsigned it = (unsigned)(r[0] & 0xffffffffull), ld = (unsigned)(r[0] >> 32);
                    ++lanes; iters += it; loads += ld; jumps += r[1] & 0xffffffffull;
                    mi = std::max(mi, it); ml = std::max(ml, ld);
                }
                wmax_inner += mi; wmax_loads += ml; busy += mi > 0;
            }
            std::fprintf(stderr, "VR_STATS %dx%dx%d flags %d: lanes %llu iters %llu jumps %llu loads %llu | "
                         "waves %zu busy %llu sum(wave max iters) %llu sum(wave max loads) %llu\n",
                         f.W, f.H, f.S, f.flags, lanes, iters, jumps, loads, nw, busy, wmax_inner, wmax_loads);
            if (const char* dump = std::getenv("VR_STATS_DUMP")) {   // per-wave records for offline analysis
                if (FILE* fp = std::fopen(dump, "wb")) {
                    std::fwrite(h.data(), 8, words, fp);
                    std::fclose(fp);
                }
            }
        }
#endif
        hip_check(launch_vrc_march(f, wc->work, nullptr, n_launch, vcls, vmaps,
                                   c->idx64 ? c->pmapx64.as<int64_t>() : nullptr, c->occ.as<uint32_t>(),
                                   c->tf_rgba.as<float4>(), (int)c->tf.size(), out, c->stream, c->batch,
                                   c->nrm.as<float>(), c->maps.as<int32_t>(),
                                   (c->leafcols ? c->occ_leafcols : c->occ_cols).as<unsigned long long>(),
                                   c->cdist_p, gtab, gtab_out, c->count_ptr));
        if (gtab_out) c->axtab[c->stream].key = std::move(pub_key);   // valid for later launches on this stream
    } else {
        if (!c->cls_test_valid) classify(c, true);
        TestFrame f = make_test(c, p, cam);
        f.out_tiles = out_tiles; f.tile_w = tile_w; f.tile_h = tile_h; f.n_work = wc->n_work; f.out_rgb = out_rgb;
        // whole frames: the work tiles off the dataset box's projection (project_box_test) are stored
        // kBgGroup per background-only workgroup, as in the VRC march
        f.bg_first = INT32_MAX;
        f.bg_group = 1;
        int n_launch = wc->n_blocks;
        if (!out_tiles && wc->bg_first >= 0 && wc->bg_first < wc->n_work) {
            f.bg_first = wc->bg_first;
            f.bg_group = kBgGroup;
            n_launch = wc->bg_first + (wc->n_work - wc->bg_first + kBgGroup - 1) / kBgGroup;
        }
        // axis views: the march axis's tables built here once per view and staged by every workgroup
        // (per stream, like the VRC view tables; a new view first drains the launches of this stream)
        const int32_t* ztab = nullptr;
        int ztab_words = 0;
        if (f.axt >= 0) {
            const bool f2b = (f.flags & 2) != 0;   // (launch_test_march's F2B)
            const bool ess = f.zero_transparent && c->tcol.p != nullptr;
            const int ax = f.axt;
            std::vector<uint32_t> key = {(uint32_t)f.S, (uint32_t)ax, (uint32_t)f2b, (uint32_t)ess, (uint32_t)f.axt_up,
                                         (uint32_t)f.tca[ax], (uint32_t)f.tnca[ax]};
            for (float v : {f.mc[10], f.mc[14], f.iv[8 + ax], f.iv[12 + ax], f.tv[5 * ax], f.tv[12 + ax],
                            ax == 0 ? f.fd1 : (ax == 1 ? f.fd2 : f.fd3)}) {
                uint32_t bits;
                std::memcpy(&bits, &v, 4);
                key.push_back(bits);
            }
            if (c->ztabs.size() >= kMaxStreamCaches && !c->ztabs.count(c->stream))   // (no sync of
                retire_stream_caches(c, nullptr);                                     //  possibly dead handles)
            vr_ctx::ZTab& zt = c->ztabs[c->stream];
            if (key != zt.key) {
                ctx_sync(c, c->stream);   // (launches reading the old table, and its upload, are done)
                zt.words = make_test_axis_table(f, f2b, ess, zt.host);
                zt.buf.ensure(zt.host.size() * sizeof(int32_t));
                hip_check(hipMemcpyAsync(zt.buf.p, zt.host.data(), zt.host.size() * sizeof(int32_t),
                                         hipMemcpyHostToDevice, c->stream));
                zt.key = std::move(key);
            }
            ztab = zt.buf.as<int32_t>();
            ztab_words = zt.words;
        }
        hip_check(launch_test_march(f, wc->work, nullptr, n_launch,
                                    c->cls_test.as<uint8_t>(), c->tf_rgba.as<float4>(), (int)c->tf.size(),
                                    c->occ_test.as<uint32_t>(), out, c->stream,
                                    c->tcol.p ? c->tcol.as<unsigned long long>() : nullptr,
                                    c->tcc.p ? c->tcc.as<uint8_t>() : nullptr,
                                    c->tcc_lay.p ? c->tcc_lay.as<int32_t>() : nullptr, c->count_ptr, ztab,
                                    ztab_words));
    }
    if (c->timing) {
        hip_check(hipEventRecord(ev.second, c->stream));
        c->ev_pending.push_back(ev);
    }
}

void render_tile_list(vr_ctx* c, const vr_params* p, const vr_camera* cam, int tile_w, int tile_h,
                      const std::vector<int32_t>& list, float* d_tiles, int out_rgb) {
    if (list.empty()) return;
    WorkCache* wc = work_for(c, p->width, p->height, tile_w, tile_h, 0, 1, &list);
    launch_frame(c, p, cam, wc, reinterpret_cast<float4*>(d_tiles), 1, tile_w, tile_h, out_rgb);
}

void assemble_slots(vr_ctx* c, int W, int H, int tile_w, int tile_h, const std::vector<int32_t>& tiles,
                    const std::vector<int32_t>& slots, int n_blocks, const float* d_tiles, const float background[4],
                    float* d_frame, int out_rgb) {
    const int ntx = (W + tile_w - 1) / tile_w, nty = (H + tile_h - 1) / tile_h;
    const size_t per = (size_t)ntx * nty;
    std::vector<int32_t> key_v(tiles);
    key_v.insert(key_v.end(), slots.begin(), slots.end());
    auto key = std::make_tuple(W, H, tile_w, tile_h, -2, n_blocks, key_v);
    auto it = c->slot_maps.find(key);
    DevBuf* map = nullptr;
    if (it != c->slot_maps.end()) {
        map = it->second.get();
    } else {
        std::vector<int32_t> slot_of(per, -1);
        for (size_t i = 0; i < tiles.size(); ++i) {
            const int32_t t = tiles[i], sl = slots[i];
            if (t < 0 || (size_t)t >= per) throw Error(VR_EINVAL, "assemble: bad tile id");
            if (sl < 0 || sl >= n_blocks) throw Error(VR_EINVAL, "assemble: bad slot");
            if (slot_of[(size_t)t] >= 0) throw Error(VR_EINVAL, "assemble: tile listed twice");
            slot_of[(size_t)t] = sl;
        }
        if (c->slot_maps.size() > 64) retire_slot_maps(c);   // (maps may be in flight)
        std::unique_ptr<DevBuf> b(new DevBuf);
        b->ensure(slot_of.size() * sizeof(int32_t));
        hip_check(hipMemcpyAsync(b->p, slot_of.data(), slot_of.size() * sizeof(int32_t), hipMemcpyHostToDevice,
                                 c->stream));
        ctx_sync(c, c->stream);   // slot_of is a host temporary
        map = b.get();
        c->slot_maps[std::move(key)] = std::move(b);
    }
    hip_check(launch_assemble_list(W, H, tile_w, tile_h, map->as<int32_t>(), reinterpret_cast<const float4*>(d_tiles),
                                   make_float4(background[0], background[1], background[2], background[3]),
                                   reinterpret_cast<float4*>(d_frame), out_rgb, c->stream));
}

void frames_in_flight(vr_ctx* c, int n, const std::function<void(int)>& launch) {
    // vr_options.frames_in_flight: 0 = one stream, k = k + 1 streams (frame f on stream f mod (k + 1))
    const int ns = std::min(std::min(n, (int)c->opt.frames_in_flight + 1), 4);
    if (ns <= 1) {
        for (int f = 0; f < n; ++f) launch(f);
        return;
    }
    if (!c->fork_ev) hip_check(hipEventCreateWithFlags(&c->fork_ev, hipEventDisableTiming));
    for (int i = 0; i < ns - 1; ++i)
        if (!c->aux_stream[i]) {
            hip_check(hipStreamCreateWithFlags(&c->aux_stream[i], hipStreamNonBlocking));
            hip_check(hipEventCreateWithFlags(&c->join_ev[i], hipEventDisableTiming));
        }
    hipStream_t main = c->stream;
    hip_check(hipEventRecord(c->fork_ev, main));
    for (int i = 0; i < ns - 1; ++i) hip_check(hipStreamWaitEvent(c->aux_stream[i], c->fork_ev, 0));
    c->batch_main = main;
    try {
        for (int f = 0; f < n; ++f) {
            const int k = f % ns;
            c->stream = k ? c->aux_stream[k - 1] : main;
            launch(f);
        }
    } catch (...) {
        c->stream = main;
        c->batch_main = nullptr;
        throw;
    }
    c->stream = main;
    c->batch_main = nullptr;
    for (int i = 0; i < ns - 1; ++i) {
        hip_check(hipEventRecord(c->join_ev[i], c->aux_stream[i]));
        hip_check(hipStreamWaitEvent(main, c->join_ev[i], 0));
    }
}

void destroy_ctx_single(vr_ctx* c) {
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (hipStream_t s : c->aux_stream)
        if (s) (void)hipStreamSynchronize(s);
    try {
        reap_retired(c, true);
    } catch (...) {
    }
    for (auto& r : c->retired)
        for (hipEvent_t e : r.ev) (void)hipEventDestroy(e);
    c->retired.clear();
    if (c->switch_ev) (void)hipEventDestroy(c->switch_ev);
    for (DevBuf* b : {&c->vol, &c->cls_vrc, &c->cls8, &c->cls_gen, &c->layout_gen, &c->pmaps_gen, &c->pmaps_pad, &c->pmaps_gen_pad, &c->cls_test, &c->maps, &c->pmaps, &c->pmapx64, &c->occ, &c->tf_rgba,
                      &c->tf_lohi, &c->alpha_nz, &c->frame, &c->counter, &c->layout, &c->egress, &c->occ_test,
                      &c->occ_cols, &c->occ_leafcols, &c->cdist, &c->nrm, &c->tcol, &c->tcc, &c->tcc_lay, &c->faces_flag})
        b->reset();
    c->work_cache.clear();
    c->slot_maps.clear();
    c->axtab.clear();
    c->ztabs.clear();
    for (auto* v : {&c->ev_free, &c->ev_pending})
        for (auto& ev : *v) { (void)hipEventDestroy(ev.first); (void)hipEventDestroy(ev.second); }
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    for (int i = 0; i < 3; ++i) {
        if (c->aux_stream[i]) (void)hipStreamDestroy(c->aux_stream[i]);
        if (c->join_ev[i]) (void)hipEventDestroy(c->join_ev[i]);
    }
    if (c->fork_ev) (void)hipEventDestroy(c->fork_ev);
    delete c;
}

void drain_timing(vr_ctx* c) {
    if (c->ev_pending.empty()) return;
    ctx_sync(c, c->stream);
    for (auto& ev : c->ev_pending) {
        float ms = 0;
        hip_check(hipEventElapsedTime(&ms, ev.first, ev.second));
        c->timing_ms += ms;
        c->timing_launches += 1;
        c->ev_free.push_back(ev);
    }
    c->ev_pending.clear();
}

}  // namespace vr

extern "C" {

int vr_api_version(void) { return VR_API_VERSION; }

const char* vr_strerror(int status) {
    switch (status) {
        case VR_OK: return "ok";
        case VR_EINVAL: return g_last_hip_error.empty() ? "invalid argument" : g_last_hip_error.c_str();
        case VR_EIO: return g_last_hip_error.empty() ? "I/O error" : g_last_hip_error.c_str();
        case VR_EFORMAT: return g_last_hip_error.empty() ? "unsupported format" : g_last_hip_error.c_str();
        case VR_ENOMEM: return "out of memory";
        case VR_EHIP: return g_last_hip_error.empty() ? "HIP error" : g_last_hip_error.c_str();
        case VR_ENODEV: return "no such GPU";
        case VR_ERANGE: return "volume or frame too large";
        case VR_ECOMM: return g_last_hip_error.empty() ? "RCCL error" : g_last_hip_error.c_str();
        default: return "unknown error";
    }
}

int vr_device_count(int32_t* count) {
    if (!count) return VR_EINVAL;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *count = n;
    return VR_OK;
}

int vr_create(const float* voxels, int64_t d1, int64_t d2, int64_t d3, double cal_max, const vr_tf_interval* tf,
              int32_t n_tf, int32_t device, vr_ctx** out) {
    if (!out) return VR_EINVAL;
    *out = nullptr;
    return guard([&] {
        *out = create_common(voxels, false, d1, d2, d3, cal_max, tf, n_tf, device, nullptr);
        return VR_OK;
    });
}

int vr_create_from_device(const float* d_voxels, int64_t d1, int64_t d2, int64_t d3, double cal_max,
                          const vr_tf_interval* tf, int32_t n_tf, int32_t device, vr_ctx** out) {
    if (!out) return VR_EINVAL;
    *out = nullptr;
    return guard([&] {
        *out = create_common(d_voxels, true, d1, d2, d3, cal_max, tf, n_tf, device, nullptr);
        return VR_OK;
    });
}

int vr_create_from_nifti(const char* path, const vr_tf_interval* tf, int32_t n_tf, int32_t device, vr_ctx** out) {
    if (!out || !path) return VR_EINVAL;
    *out = nullptr;
    return guard([&] {
        NiftiFile nf(path);
        *out = create_common(nf.volume.data(), false, nf.header.dim[1], nf.header.dim[2], nf.header.dim[3],
                             nf.header.cal_max, tf, n_tf, device, nullptr);
        return VR_OK;
    });
}

int vr_options_default(vr_options* o) {
    if (!o) return VR_EINVAL;
    std::memset(o, 0, sizeof *o);
    o->brick[0] = 4; o->brick[1] = 4; o->brick[2] = 8;
    o->cell_shift = -1;
    o->force_idx64 = 0;
    o->batch = 0;
    o->cull = 2;
    o->view_table_reuse = 1;
    o->work_order = 0;
    o->axis_table = 1;
    o->occ_lds = 1;
    o->persist_wgs = 0;
    o->farm_tile = 64;
    o->farm_rank0_weight = 1.0f;
    o->leaf_map_pad = 1;
    o->exact_skip = 1;
    o->frames_in_flight = 1;
    o->test_plane_march = 1;
    o->comm_timeout_ms = 60000;
    o->class_bits = 0;
    o->run_words = 0;
    o->table_split = 1;
    // x-major (round 6): with the plane table the bricked layout's three offset-table reads per sample
    // cost more than its traffic saves -- C3 TEST oblique ESS + ERT 0.205 -> 0.191 ms one launch at a
    // time, ESS 0.46 -> 0.43 ms (profiles/r6_ab/ab2_*.log); round 5 chose 3 (82 -> 18 MB past L2 per
    // launch at the same frame time, before the plane table)
    o->test_corners = 0;
    o->leaf_columns = 1;   // C3 default view
    return VR_OK;
}

int vr_create_ex(const float* voxels, int32_t voxels_on_device, int64_t d1, int64_t d2, int64_t d3, double cal_max,
                 const vr_tf_interval* tf, int32_t n_tf, int32_t device, const vr_options* opt, vr_ctx** out) {
    if (!out) return VR_EINVAL;
    *out = nullptr;
    return guard([&] {
        *out = create_common(voxels, voxels_on_device != 0, d1, d2, d3, cal_max, tf, n_tf, device, opt);
        return VR_OK;
    });
}

int vr_get_options(vr_ctx* c, vr_options* o) {
    if (!c || !o) return VR_EINVAL;
    *o = c->opt;
    return VR_OK;
}

int vr_set_options(vr_ctx* c, const vr_options* o) {
    if (!c || !o) return VR_EINVAL;
    return guard([&] {
        check_options(*o);
        const vr_options& cur = c->opt;
        if (o->brick[0] != cur.brick[0] || o->brick[1] != cur.brick[1] || o->brick[2] != cur.brick[2] ||
            o->cell_shift != cur.cell_shift || o->force_idx64 != cur.force_idx64 || o->class_bits != cur.class_bits ||
            o->test_corners != cur.test_corners || o->leaf_columns != cur.leaf_columns)
            throw Error(VR_EINVAL,
                        "vr_set_options: brick / cell_shift / force_idx64 / class_bits / test_corners / leaf_columns are fixed at vr_create_ex");
        group_for_each(c, [](vr_ctx* pc, void* a) { apply_render_options(pc, *static_cast<const vr_options*>(a)); },
                       const_cast<vr_options*>(o));
        group_options_changed(c);
        return VR_OK;
    });
}

int vr_set_transfer_function(vr_ctx* c, const vr_tf_interval* tf, int32_t n_tf) {
    if (!c) return VR_EINVAL;
    return guard([&] {
        set_tf(c, tf, n_tf);   // validates before any part changes
        struct A { const vr_tf_interval* tf; int32_t n; } a{tf, n_tf};
        group_for_each(c, [](vr_ctx* pc, void* p) {
            const A* x = static_cast<const A*>(p);
            set_device(pc);
            set_tf(pc, x->tf, x->n);
            classify(pc, pc->cls_test_valid);
        }, &a);
        return VR_OK;
    });
}

int vr_destroy(vr_ctx* c) {
    if (!c) return VR_OK;
    if (c->group) {   // the other devices' parts and the communicators first
        group_destroy(c->group);
        c->group = nullptr;
    }
    destroy_ctx_single(c);
    return VR_OK;
}

int vr_render(vr_ctx* c, const vr_params* p, const vr_camera* cam, float* out, int32_t out_flags) {
    if (!c || !cam) return VR_EINVAL;
    if (c->group) {   // multi-GPU context: tiles farmed over its devices, frame assembled on the first
        return guard([&] {
            check_params(p);
            group_render(c, p, cam, 1, out, out_flags);
            return VR_OK;
        });
    }
    if (!out) return VR_EINVAL;
    return guard([&] {
        const bool out_on_device = (out_flags & VR_OUT_DEVICE) != 0;
        check_params(p);
        set_device(c);
        // whole-frame culling: work tiles off the projected dataset box are background-filled
        TileRect rect;
        if (c->cull) rect = visible_rect(c, p, cam, kWgRaysX, kWgRaysY);
        WorkCache* wc = c->order_mode == 0 ? frame_list(c, p, cam, rect)
                                           : work_for(c, p->width, p->height, 0, 0, 0, 1, nullptr, &rect);
        const size_t bytes = (size_t)p->width * p->height * sizeof(float4);
        float4* dst;
        if (out_on_device) {
            dst = reinterpret_cast<float4*>(out);
        } else {
            c->frame.ensure(bytes);
            dst = c->frame.as<float4>();
        }
        launch_frame(c, p, cam, wc, dst, 0, 0, 0);
        if (!out_on_device) {
            hip_check(hipMemcpyAsync(out, dst, bytes, hipMemcpyDeviceToHost, c->stream));
            hip_check(hipStreamSynchronize(c->stream));
        } else if (!(out_flags & VR_OUT_ASYNC)) {
            hip_check(hipStreamSynchronize(c->stream));
        }
        return VR_OK;
    });
}

int vr_render_batch(vr_ctx* c, const vr_params* p, const vr_camera* cams, int32_t n_frames, float* out,
                    int32_t out_flags) {
    if (!c || !cams || n_frames <= 0) return VR_EINVAL;
    return guard([&] {
        check_params(p);
        if (c->group) {
            group_render(c, p, cams, n_frames, out, out_flags);
            return VR_OK;
        }
        if (!out) throw Error(VR_EINVAL, "vr_render_batch: no output");
        const size_t fpx = (size_t)p->width * p->height * 4;
        const bool dev = (out_flags & VR_OUT_DEVICE) != 0;
        if (!dev) {   // host output: frame by frame, each copied out
            for (int32_t f = 0; f < n_frames; ++f) {
                const int rc = vr_render(c, p, &cams[f], out + (size_t)f * fpx, 0);
                if (rc < 0) return rc;
            }
            return VR_OK;
        }
        set_device(c);
        frames_in_flight(c, n_frames, [&](int f) {
            TileRect rect;
            if (c->cull) rect = visible_rect(c, p, &cams[f], kWgRaysX, kWgRaysY);
            WorkCache* wc = c->order_mode == 0 ? frame_list(c, p, &cams[f], rect)
                                               : work_for(c, p->width, p->height, 0, 0, 0, 1, nullptr, &rect);
            launch_frame(c, p, &cams[f], wc, reinterpret_cast<float4*>(out + (size_t)f * fpx), 0, 0, 0);
        });
        if (!(out_flags & VR_OUT_ASYNC)) hip_check(hipStreamSynchronize(c->stream));
        return VR_OK;
    });
}

int vr_render_tiles(vr_ctx* c, const vr_params* p, const vr_camera* cam, int32_t tile_w, int32_t tile_h,
                    int32_t first_tile, int32_t tile_stride, float* d_tiles, int32_t* n_tiles_out,
                    int32_t out_flags) {
    if (!c || !cam || !d_tiles) return VR_EINVAL;
    return guard([&] {
        check_params(p);
        if (tile_w <= 0 || tile_h <= 0 || tile_w % kWgRaysX || tile_h % kWgRaysY || tile_w > 32768 || tile_h > 32768)
            throw Error(VR_EINVAL, "vr_render_tiles: tile sizes must be positive multiples of 16");
        if (first_tile < 0 || tile_stride <= 0) throw Error(VR_EINVAL, "vr_render_tiles: bad first/stride");
        set_device(c);
        WorkCache* wc = work_for(c, p->width, p->height, tile_w, tile_h, first_tile, tile_stride);
        const int ntx = (p->width + tile_w - 1) / tile_w, nty = (p->height + tile_h - 1) / tile_h;
        const int64_t nt = (int64_t)ntx * nty;
        const int mine = first_tile >= nt ? 0 : (int)((nt - 1 - first_tile) / tile_stride + 1);
        if (n_tiles_out) *n_tiles_out = mine;
        launch_frame(c, p, cam, wc, reinterpret_cast<float4*>(d_tiles), 1, tile_w, tile_h, (out_flags & VR_OUT_RGB) ? 1 : 0);
        if (!(out_flags & VR_OUT_ASYNC)) hip_check(hipStreamSynchronize(c->stream));
        return VR_OK;
    });
}

int vr_visible_tiles(vr_ctx* c, const vr_params* p, const vr_camera* cam, int32_t tile_w, int32_t tile_h,
                     int32_t* tiles, int32_t capacity, int32_t* n_out) {
    if (!c || !cam || !n_out || tile_w <= 0 || tile_h <= 0 || capacity < 0) return VR_EINVAL;
    return guard([&] {
        check_params(p);
        const std::vector<int32_t> v = visible_tiles(c, p, cam, tile_w, tile_h);
        *n_out = (int32_t)v.size();
        if (tiles) std::copy(v.begin(), v.begin() + std::min<size_t>(v.size(), (size_t)capacity), tiles);
        return VR_OK;
    });
}

int vr_render_tile_list(vr_ctx* c, const vr_params* p, const vr_camera* cam, int32_t tile_w, int32_t tile_h,
                        const int32_t* tiles, int32_t n_tiles, int32_t first, int32_t stride, float* d_tiles,
                        int32_t* n_tiles_out, int32_t out_flags) {
    if (!c || !cam || !d_tiles || n_tiles < 0 || (n_tiles > 0 && !tiles)) return VR_EINVAL;
    return guard([&] {
        check_params(p);
        if (tile_w <= 0 || tile_h <= 0 || tile_w % kWgRaysX || tile_h % kWgRaysY || tile_w > 32768 || tile_h > 32768)
            throw Error(VR_EINVAL, "vr_render_tile_list: tile sizes must be positive multiples of 16");
        if (first < 0 || stride <= 0) throw Error(VR_EINVAL, "vr_render_tile_list: bad first/stride");
        const int ntx = (p->width + tile_w - 1) / tile_w, nty = (p->height + tile_h - 1) / tile_h;
        std::vector<int32_t> list(tiles, tiles + n_tiles);
        for (int32_t t : list)
            if (t < 0 || t >= ntx * nty) throw Error(VR_EINVAL, "vr_render_tile_list: tile id out of range");
        set_device(c);
        WorkCache* wc = work_for(c, p->width, p->height, tile_w, tile_h, first, stride, &list);
        const int mine = first >= n_tiles ? 0 : (n_tiles - 1 - first) / stride + 1;
        if (n_tiles_out) *n_tiles_out = mine;
        launch_frame(c, p, cam, wc, reinterpret_cast<float4*>(d_tiles), 1, tile_w, tile_h, (out_flags & VR_OUT_RGB) ? 1 : 0);
        if (!(out_flags & VR_OUT_ASYNC)) hip_check(hipStreamSynchronize(c->stream));
        return VR_OK;
    });
}

int vr_assemble_tile_list(vr_ctx* c, int32_t W, int32_t H, int32_t tile_w, int32_t tile_h, const int32_t* tiles,
                          int32_t n_tiles, int32_t n_ranks, int32_t max_tiles, const float* d_tiles,
                          const float background[4], float* d_frame, int32_t out_flags) {
    if (!c || !d_frame || !background || W <= 0 || H <= 0 || tile_w <= 0 || tile_h <= 0 || n_ranks <= 0 ||
        max_tiles < 0 || n_tiles < 0 || (n_tiles > 0 && (!tiles || !d_tiles)))
        return VR_EINVAL;
    return guard([&] {
        const int ntx = (W + tile_w - 1) / tile_w, nty = (H + tile_h - 1) / tile_h;
        if ((int64_t)(n_tiles + n_ranks - 1) / n_ranks > max_tiles)
            throw Error(VR_EINVAL, "vr_assemble_tile_list: max_tiles_per_rank too small for the list");
        std::vector<int32_t> list(tiles, tiles + n_tiles);
        auto key = std::make_tuple(W, H, tile_w, tile_h, n_ranks, max_tiles, list);
        auto it = c->slot_maps.find(key);
        DevBuf* map = nullptr;
        set_device(c);
        if (it != c->slot_maps.end()) {
            map = it->second.get();
        } else {
            std::vector<int32_t> slot_of((size_t)ntx * nty, -1);
            for (int32_t i = 0; i < n_tiles; ++i) {   // tile list[r + k*N] is block k of rank r
                if (list[i] < 0 || list[i] >= ntx * nty) throw Error(VR_EINVAL, "vr_assemble_tile_list: bad tile id");
                slot_of[(size_t)list[i]] = (i % n_ranks) * max_tiles + i / n_ranks;
            }
            if (c->slot_maps.size() > 64) retire_slot_maps(c);   // (maps may be in flight)
            std::unique_ptr<DevBuf> b(new DevBuf);
            b->ensure(slot_of.size() * sizeof(int32_t));
            hip_check(hipMemcpy(b->p, slot_of.data(), slot_of.size() * sizeof(int32_t), hipMemcpyHostToDevice));
            map = b.get();
            c->slot_maps[std::move(key)] = std::move(b);
        }
        hip_check(launch_assemble_list(W, H, tile_w, tile_h, map->as<int32_t>(),
                                       reinterpret_cast<const float4*>(d_tiles),
                                       make_float4(background[0], background[1], background[2], background[3]),
                                       reinterpret_cast<float4*>(d_frame), (out_flags & VR_OUT_RGB) ? 1 : 0, c->stream));
        if (!(out_flags & VR_OUT_ASYNC)) hip_check(hipStreamSynchronize(c->stream));
        return VR_OK;
    });
}

int vr_assemble_tile_slots_multi(vr_ctx* c, int32_t W, int32_t H, int32_t tile_w, int32_t tile_h,
                                 const int32_t* tiles, const int32_t* slots, int32_t n_tiles, int32_t n_frames,
                                 int32_t n_blocks, const float* d_tiles, const float background[4], float* d_frames,
                                 int32_t out_flags) {
    if (!c || !d_frames || !background || W <= 0 || H <= 0 || tile_w <= 0 || tile_h <= 0 || n_blocks < 0 ||
        n_tiles < 0 || n_frames <= 0 || (n_tiles > 0 && (!tiles || !slots || !d_tiles)))
        return VR_EINVAL;
    return guard([&] {
        const int ntx = (W + tile_w - 1) / tile_w, nty = (H + tile_h - 1) / tile_h;
        const size_t per = (size_t)ntx * nty;
        std::vector<int32_t> key_v(tiles, tiles + n_tiles);
        key_v.insert(key_v.end(), slots, slots + (size_t)n_tiles * n_frames);
        auto key = std::make_tuple(W, H, tile_w, tile_h, -1 - n_frames, n_blocks, key_v);
        auto it = c->slot_maps.find(key);
        DevBuf* map = nullptr;
        set_device(c);
        if (it != c->slot_maps.end()) {
            map = it->second.get();
        } else {
            std::vector<int32_t> slot_of(per * n_frames, -1);
            for (int32_t f = 0; f < n_frames; ++f)
                for (int32_t i = 0; i < n_tiles; ++i) {
                    const int32_t t = tiles[i], sl = slots[(size_t)f * n_tiles + i];
                    if (t < 0 || (size_t)t >= per) throw Error(VR_EINVAL, "vr_assemble_tile_slots: bad tile id");
                    if (sl < 0 || sl >= n_blocks) throw Error(VR_EINVAL, "vr_assemble_tile_slots: bad slot");
                    if (slot_of[f * per + t] >= 0) throw Error(VR_EINVAL, "vr_assemble_tile_slots: tile listed twice");
                    slot_of[f * per + t] = sl;
                }
            if (c->slot_maps.size() > 64) retire_slot_maps(c);   // (maps may be in flight)
            std::unique_ptr<DevBuf> b(new DevBuf);
            b->ensure(slot_of.size() * sizeof(int32_t));
            hip_check(hipMemcpy(b->p, slot_of.data(), slot_of.size() * sizeof(int32_t), hipMemcpyHostToDevice));
            map = b.get();
            c->slot_maps[std::move(key)] = std::move(b);
        }
        hip_check(launch_assemble_list(W, H, tile_w, tile_h, map->as<int32_t>(),
                                       reinterpret_cast<const float4*>(d_tiles),
                                       make_float4(background[0], background[1], background[2], background[3]),
                                       reinterpret_cast<float4*>(d_frames), (out_flags & VR_OUT_RGB) ? 1 : 0, c->stream,
                                       n_frames));
        if (!(out_flags & VR_OUT_ASYNC)) hip_check(hipStreamSynchronize(c->stream));
        return VR_OK;
    });
}

int vr_assemble_tile_slots(vr_ctx* c, int32_t W, int32_t H, int32_t tile_w, int32_t tile_h, const int32_t* tiles,
                           const int32_t* slots, int32_t n_tiles, int32_t n_blocks, const float* d_tiles,
                           const float background[4], float* d_frame, int32_t out_flags) {
    return vr_assemble_tile_slots_multi(c, W, H, tile_w, tile_h, tiles, slots, n_tiles, 1, n_blocks, d_tiles,
                                        background, d_frame, out_flags);
}

int vr_assemble_tiles(vr_ctx* c, int32_t W, int32_t H, int32_t tile_w, int32_t tile_h, int32_t n_ranks,
                      int32_t max_tiles, const float* d_tiles, float* d_frame, int32_t out_flags) {
    if (!c || !d_tiles || !d_frame || W <= 0 || H <= 0 || tile_w <= 0 || tile_h <= 0 || n_ranks <= 0 || max_tiles < 0)
        return VR_EINVAL;
    return guard([&] {
        set_device(c);
        hip_check(launch_assemble(W, H, tile_w, tile_h, n_ranks, max_tiles, reinterpret_cast<const float4*>(d_tiles),
                                  reinterpret_cast<float4*>(d_frame), (out_flags & VR_OUT_RGB) ? 1 : 0, c->stream));
        if (!(out_flags & VR_OUT_ASYNC)) hip_check(hipStreamSynchronize(c->stream));
        return VR_OK;
    });
}

int vr_count_samples(vr_ctx* c, const vr_params* p, const vr_camera* cam, uint64_t* n_in) {
    if (!c || !cam || !n_in) return VR_EINVAL;
    return guard([&] {
        check_params(p);
        set_device(c);
        WorkCache* wc = work_for(c, p->width, p->height, 0, 0, 0, 1);
        VrcFrame f = make_vrc(c, p, cam);
        f.n_work = wc->n_work;
        hip_check(hipMemsetAsync(c->counter.p, 0, 8, c->stream));
        if (wc->n_work)
            hip_check(launch_vrc_count(f, wc->work.as<WorkTile>(), wc->n_work, c->maps.as<int32_t>(),
                                       c->counter.as<unsigned long long>(), c->stream));
        unsigned long long h = 0;
        hip_check(hipMemcpyAsync(&h, c->counter.p, 8, hipMemcpyDeviceToHost, c->stream));
        hip_check(hipStreamSynchronize(c->stream));
        *n_in = h;
        return VR_OK;
    });
}

int vr_count_work(vr_ctx* c, const vr_params* p, const vr_camera* cam, vr_work_count* out) {
    if (!c || !cam || !out) return VR_EINVAL;
    return guard([&] {
        check_params(p);
        set_device(c);
        group_check_alive(c);   // a failed multi-GPU context fails here with VR_ECOMM, as vr_render does
        // the whole frame on this context's GPU (a multi-GPU context's first part), through the same
        // work list, options and kernel variant as vr_render, in the counting instantiation
        TileRect rect;
        if (c->cull) rect = visible_rect(c, p, cam, kWgRaysX, kWgRaysY);
        WorkCache* wc = c->order_mode == 0 ? frame_list(c, p, cam, rect)
                                           : work_for(c, p->width, p->height, 0, 0, 0, 1, nullptr, &rect);
        c->frame.ensure((size_t)p->width * p->height * sizeof(float4));
        hip_check(hipMemsetAsync(c->counter.p, 0, 24, c->stream));
        c->count_ptr = c->counter.as<unsigned long long>();
        try {
            launch_frame(c, p, cam, wc, c->frame.as<float4>(), 0, 0, 0);
        } catch (...) {
            c->count_ptr = nullptr;
            throw;
        }
        c->count_ptr = nullptr;
        unsigned long long h[3] = {0, 0, 0};
        hip_check(hipMemcpyAsync(h, c->counter.p, 24, hipMemcpyDeviceToHost, c->stream));
        ctx_sync(c, c->stream);   // (a part of a multi-GPU context: polled, bounded, VR_ECOMM on a failed group)
        out->gathers = h[0];
        out->samples = h[1];
        out->bytes = h[2];
        out->reserved = 0;
        return VR_OK;
    });
}

int vr_count_marched(vr_ctx* c, const vr_params* p, const vr_camera* cam, uint64_t* gathers, uint64_t* samples) {
    if (!c || !cam || !gathers) return VR_EINVAL;
    if (p && p->mode != VR_MODE_VRC) return VR_EINVAL;   // (VRC frames: the 1-byte gathers it reports)
    vr_work_count w;
    const int rc = vr_count_work(c, p, cam, &w);
    if (rc == VR_OK) {
        *gathers = w.gathers;
        if (samples) *samples = w.samples;
    }
    return rc;
}

int vr_frame_to_rgb8(vr_ctx* c, int32_t W, int32_t H, int32_t orientation, const float* d_frame, uint8_t* rgb,
                     int32_t out_flags) {
    if (!c || !d_frame || !rgb || W <= 0 || H <= 0) return VR_EINVAL;
    if (orientation < VR_ORIENT_RAW || orientation > VR_ORIENT_TEST_DISPLAY) return VR_EINVAL;
    return guard([&] {
        set_device(c);
        const size_t bytes = (size_t)W * H * 3;
        uint8_t* dst = rgb;
        if (!(out_flags & VR_OUT_DEVICE)) {
            c->egress.ensure(bytes);
            dst = c->egress.as<uint8_t>();
        }
        hip_check(launch_egress(reinterpret_cast<const float4*>(d_frame), dst, W, H, orientation, c->stream));
        if (!(out_flags & VR_OUT_DEVICE))
            hip_check(hipMemcpyAsync(rgb, dst, bytes, hipMemcpyDeviceToHost, c->stream));
        if (!(out_flags & VR_OUT_ASYNC) || !(out_flags & VR_OUT_DEVICE)) hip_check(hipStreamSynchronize(c->stream));
        return VR_OK;
    });
}

int vr_render_png(vr_ctx* c, const vr_params* p, const vr_camera* cam, int32_t orientation, const char* path) {
    if (!c || !p || !cam || !path) return VR_EINVAL;
    if (orientation < VR_ORIENT_RAW || orientation > VR_ORIENT_TEST_DISPLAY) return VR_EINVAL;
    return guard([&] {
        check_params(p);
        set_device(c);
        const size_t px = (size_t)p->width * p->height;
        DevBuf frame;   // own buffer: c->frame is vr_render's host-output staging
        frame.ensure(px * sizeof(float4));
        int rc = vr_render(c, p, cam, frame.as<float>(), VR_OUT_DEVICE);
        if (rc < 0) return rc;
        std::vector<uint8_t> rgb(px * 3);
        rc = vr_frame_to_rgb8(c, p->width, p->height, orientation, frame.as<float>(), rgb.data(), 0);
        if (rc < 0) return rc;
        return vr_write_png(path, p->width, p->height, rgb.data());
    });
}

int vr_point_cloud(vr_ctx* c, float* d_out, int32_t out_flags) {
    if (!c || !d_out) return VR_EINVAL;
    return guard([&] {
        set_device(c);
        const int n_tf = (int)c->tf.size();
        hip_check(launch_point(c->vol.as<float>(), c->d[0], c->d[1], c->d[2], c->cal_max, c->tf_lohi.as<float>(),
                               c->tf_lohi.as<float>() + n_tf, n_tf, c->tf_rgba.as<float4>(), d_out, c->stream));
        if (!(out_flags & VR_OUT_ASYNC)) hip_check(hipStreamSynchronize(c->stream));
        return VR_OK;
    });
}

int vr_write_png(const char* path, int32_t W, int32_t H, const uint8_t* rgb) {
    if (!path || !rgb || W <= 0 || H <= 0) return VR_EINVAL;
    return guard([&] {
        try {
            write_png_rgb8(path, W, H, rgb);
        } catch (const std::runtime_error& e) {
            throw Error(VR_EIO, e.what());
        }
        return VR_OK;
    });
}

int vr_synthetic_volume(float* d_out, int64_t n, int64_t x0, int64_t nx, uint64_t seed, int32_t device,
                        void* hip_stream) {
    if (!d_out || n <= 0 || x0 < 0 || nx < 0 || x0 + nx > n) return VR_EINVAL;
    return guard([&] {
        int ndev = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) throw Error(VR_ENODEV, "vr_synthetic_volume: no GPU");
        if (device < 0 || device >= ndev) throw Error(VR_ENODEV, "vr_synthetic_volume: bad device index");
        hip_check(hipSetDevice(device));
        hipStream_t st = static_cast<hipStream_t>(hip_stream);
        hip_check(launch_synthetic(d_out, n, x0, nx, seed, st));
        hip_check(hipStreamSynchronize(st));
        return VR_OK;
    });
}

int vr_synchronize(vr_ctx* c) {
    if (!c) return VR_EINVAL;
    return guard([&] {
        if (c->group) {
            group_sync(c);
        } else {
            set_device(c);
            hip_check(hipStreamSynchronize(c->stream));
        }
        return VR_OK;
    });
}

int vr_set_stream(vr_ctx* c, void* s) {
    if (!c) return VR_EINVAL;
    return guard([&] {
        if (!s && !c->own_stream) {   // back to the context's own stream after releasing it (below)
            set_device(c);
            hip_check(hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking));
        }
        hipStream_t ns = s ? static_cast<hipStream_t>(s) : c->own_stream;   // (view tables are kept per stream)
        if (ns != c->stream) {
            // the new stream starts after everything queued on the old one: the context's launches stay
            // ordered on its current stream (cache buffers are retired behind one event there)
            set_device(c);
            if (!c->switch_ev) hip_check(hipEventCreateWithFlags(&c->switch_ev, hipEventDisableTiming));
            hip_check(hipEventRecord(c->switch_ev, c->stream));
            hip_check(hipStreamWaitEvent(ns, c->switch_ev, 0));
        }
        const hipStream_t prev = c->stream;
        c->stream = ns;
        if (s && c->own_stream && prev == c->own_stream && !c->group) {
            // A caller's stream replaces the context's own, which is released: HIP gives a process a few
            // hardware queues (GPU_MAX_HW_QUEUES, 4 by default) and shares them among streams beyond
            // that, so an idle own stream still holds a share -- a second context's frames-in-flight
            // stream then landed on the caller's queue and its two frames in flight ran one after the
            // other (C4 timed after a C3 context: 48.1 against 58.2 G rays/s alone; 55.1 with 8 queues).
            // Its view table, work list and TEST axis table are retired with it (a later stream may
            // reuse the handle); the stream is destroyed behind its queued work (the switch event above
            // orders the new stream after it).
            retire_stream_caches(c, &prev);
            hip_check(hipStreamDestroy(prev));
            c->own_stream = nullptr;
        }
        return VR_OK;
    });
}

int vr_params_default(int32_t W, int32_t H, int32_t S, vr_params* out) {
    if (!out || W <= 0 || H <= 0 || S <= 0) return VR_EINVAL;
    std::memset(out, 0, sizeof *out);
    out->width = W; out->height = H; out->samples_per_ray = S;
    out->mode = VR_MODE_VRC; out->flags = 0;
    default_screen(W, H, S, &out->real_screen_width, &out->real_screen_height, &out->viewplane_distance,
                   &out->front_clip_plane, &out->sample_distance);
    out->background[0] = 0.2f; out->background[1] = 0.2f; out->background[2] = 0.2f; out->background[3] = 1.0f;
    out->ert_epsilon = 1e-5f;
    out->shade_ambient = 0.3f; out->shade_diffuse = 0.7f; out->shade_specular = 0.2f; out->shade_shininess = 16.0f;
    return VR_OK;
}

static void put(const CameraState& cs, vr_camera* out) {
    const glmf::vec3* v[5] = {&cs.pos, &cs.front, &cs.right, &cs.up, &cs.top_left};
    float* o[5] = {out->pos, out->front, out->right, out->up, out->top_left};
    for (int i = 0; i < 5; ++i) { o[i][0] = v[i]->x; o[i][1] = v[i]->y; o[i][2] = v[i]->z; }
}

int vr_camera_derive(const float pos[3], const float up[3], float rsw, float rsh, vr_camera* out) {
    if (!pos || !up || !out) return VR_EINVAL;
    put(derive_camera({pos[0], pos[1], pos[2]}, {up[0], up[1], up[2]}, rsw, rsh), out);
    return VR_OK;
}

int vr_camera_derive_conic(const float pos[3], const float up[3], float rsw, float rsh, float vpd, vr_camera* out) {
    if (!pos || !up || !out) return VR_EINVAL;
    put(derive_camera_conic({pos[0], pos[1], pos[2]}, {up[0], up[1], up[2]}, rsw, rsh, vpd), out);
    return VR_OK;
}

int vr_camera_default(int32_t W, int32_t H, vr_camera* out) {
    if (!out || W <= 0 || H <= 0) return VR_EINVAL;
    put(default_camera(W, H), out);
    return VR_OK;
}

int vr_camera_reset(vr_camera* out) {
    if (!out) return VR_EINVAL;
    put(reset_camera(), out);
    return VR_OK;
}

int vr_default_transfer_function(vr_tf_interval* out, int32_t capacity) {
    TransferFunction t;
    if (!out || capacity < t.size()) return VR_EINVAL;
    for (int i = 0; i < t.size(); ++i) {
        out[i].lo = t.material_intervals[i].lower_bound;
        out[i].hi = t.material_intervals[i].higher_bound;
        std::memcpy(out[i].rgba, t.material_intervals[i].material.color, 16);
    }
    return t.size();
}

int vr_nifti_read(const char* path, int64_t dims[3], double* cal_max, float* voxels) {
    if (!path || !dims || !cal_max) return VR_EINVAL;
    return guard([&] {
        NiftiFile nf(path);
        for (int i = 0; i < 3; ++i) dims[i] = nf.header.dim[i + 1];
        *cal_max = nf.header.cal_max;
        if (voxels) std::memcpy(voxels, nf.volume.data(), nf.volume.size() * sizeof(float));
        return VR_OK;
    });
}

int vr_octree_leaf_maps(int64_t d1, int64_t d2, int64_t d3, int32_t* maps, int64_t capacity, uint32_t* depth) {
    if (d1 <= 0 || d2 <= 0 || d3 <= 0) return VR_EINVAL;
    return guard([&] {
        OctreeHandler o;
        o.build(d1, d2, d3);
        if (depth) *depth = o.maximum_depth;
        if (maps && capacity >= (int64_t)o.maps.size()) std::memcpy(maps, o.maps.data(), o.maps.size() * 4);
        return (int)o.maps.size();
    });
}

int vr_get_volume_info(vr_ctx* c, vr_volume_info* out) {
    if (!c || !out) return VR_EINVAL;
    std::memset(out, 0, sizeof *out);
    for (int i = 0; i < 3; ++i) out->dim[i] = c->d[i];
    out->cal_max = c->cal_max;
    out->longest_dimension = c->oct.longest_dimension;
    out->octree_depth = c->oct.maximum_depth;
    out->n_tf = (int32_t)c->tf.size();
    out->zero_transparent = c->zero_transparent;
    uint64_t b = 0;
    for (DevBuf* d : {&c->vol, &c->cls_vrc, &c->cls8, &c->cls_gen, &c->layout_gen, &c->pmaps_gen, &c->pmaps_pad, &c->pmaps_gen_pad, &c->cls_test, &c->maps, &c->pmaps, &c->pmapx64, &c->occ, &c->tf_rgba,
                      &c->tf_lohi, &c->alpha_nz, &c->frame, &c->counter, &c->layout, &c->egress, &c->occ_test, &c->occ_cols, &c->occ_leafcols, &c->cdist, &c->nrm, &c->tcol, &c->tcc, &c->tcc_lay})
        b += d->bytes;
    out->device_bytes = b;
    out->idx64 = c->idx64 ? 1 : 0;
    out->reserved = 0;
    out->class_bytes = (uint64_t)c->cls_bytes;
    return VR_OK;
}

int vr_timing_enable(vr_ctx* c, int32_t enable) {
    if (!c) return VR_EINVAL;
    return guard([&] {
        // every GPU of a one-process group (vr_group_timing_read reads each part)
        group_for_each(c, [](vr_ctx* pc, void* e) { pc->timing = *static_cast<int32_t*>(e) != 0; }, &enable);
        return VR_OK;
    });
}

int vr_timing_read(vr_ctx* c, double* total_ms, int64_t* launches, int32_t reset) {
    if (!c) return VR_EINVAL;
    return guard([&] {
        set_device(c);
        drain_timing(c);
        if (total_ms) *total_ms = c->timing_ms;
        if (launches) *launches = c->timing_launches;
        if (reset) { c->timing_ms = 0; c->timing_launches = 0; }
        return VR_OK;
    });
}

}  // extern "C"
