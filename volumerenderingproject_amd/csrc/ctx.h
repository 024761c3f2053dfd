// ctx.h -- internal: the context object behind the C-ABI and the helpers vr_api.cpp and
// vr_multi.cpp share.  Not part of the ABI (include/vr_api.h).
#pragma once
#include <hip/hip_runtime.h>

#include <functional>
#include <map>
#include <memory>
#include <string>
#include <tuple>
#include <utility>
#include <vector>

#include "../../include/vr_api.h"
#include "host/scene.h"
#include "vr_device.h"

namespace vr {

extern thread_local std::string g_last_hip_error;

struct HipFail {
    hipError_t e;
};
inline void hip_check(hipError_t e) {
    if (e != hipSuccess) {
        g_last_hip_error = hipGetErrorString(e);
        throw HipFail{e};
    }
}

template <class F> int guard(F&& f) {
    try {
        return f();
    } catch (const Error& e) {
        g_last_hip_error = e.what();
        return e.code;
    } catch (const HipFail&) {
        return VR_EHIP;
    } catch (const std::bad_alloc&) {
        return VR_ENOMEM;
    } catch (...) {
        return VR_EINVAL;
    }
}

struct DevBuf {   // owning device allocation (freed on destruction: contexts, tile caches)
    void* p = nullptr;
    size_t bytes = 0;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    void swap(DevBuf& o) {
        std::swap(p, o.p);
        std::swap(bytes, o.bytes);
    }
    ~DevBuf() { reset(); }
    void reset() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    void ensure(size_t n) {
        if (n <= bytes && p) return;
        reset();
        hipError_t e = hipMalloc(&p, n ? n : 16);
        if (e != hipSuccess) {
            p = nullptr;
            if (e == hipErrorOutOfMemory) throw Error(VR_ENOMEM, "hipMalloc failed");
            hip_check(e);
        }
        bytes = n;
    }
    template <class T> T* as() const { return static_cast<T*>(p); }
};

struct TileRect {   // visible_rect's result
    int tx0 = 0, tx1 = -1, ty0 = 0, ty1 = -1;   // inclusive tile ranges; empty when tx1 < tx0
    bool all = true;
};

struct WorkCache {
    DevBuf work;   // WorkTiles in dispatch order (culled whole-frame tiles last, slot = -1)
    int n_work = 0, n_blocks = 0;
    int bg_first = -1;   // first culled entry (-1: none / not a whole-frame list)
};

// A work list in device memory the caller keeps alive (multi-GPU plans built on the device)
struct WorkView {
    const WorkTile* work = nullptr;
    int n_work = 0, n_blocks = 0;
    int bg_first = -1;
};

struct Group;   // multi-GPU state of a context (vr_multi.cpp)

// Device buffers evicted from a cache while launches queued on the ctx stream may still read them:
// freed once an event recorded behind that work has completed (no host or device-wide drain).
struct Retired {
    std::vector<hipEvent_t> ev;   // one per stream the context may have queued readers on
    std::vector<std::unique_ptr<DevBuf>> bufs;
    std::vector<std::vector<int32_t>> hosts;   // host sources of uploads that may still be in flight
};

}  // namespace vr

struct vr_ctx {
    int device = 0;
    hipStream_t own_stream = nullptr, stream = nullptr;
    hipStream_t aux_stream[3] = {nullptr, nullptr, nullptr};   // frames in flight: frame f of a batch on
                                                        //   stream f mod n (0 = `stream`, i = aux_stream[i - 1])
    hipStream_t batch_main = nullptr;                   //   (the ctx stream while a batch alternates c->stream)
    hipEvent_t fork_ev = nullptr, join_ev[3] = {nullptr, nullptr, nullptr};   //   forked from / joined into `stream`
    int64_t d[3] = {0, 0, 0};
    double cal_max = 0;
    int max_intensity = 0;
    vr::OctreeHandler oct;
    vr::DevBuf vol, cls_vrc, cls_test, maps, pmaps, pmapx64, occ, tf_rgba, tf_lohi, alpha_nz, frame, counter, layout, egress, occ_test, occ_cols, occ_leafcols, cdist, nrm;
    const uint8_t* cdist_p = nullptr;   // the settled buffer of the two in cdist
    int tcb = 3, tnc[3] = {0, 0, 0};   // TEST macro cells
    vr::DevBuf tcc, tcc_lay;             // TEST general views: the 8 corner classes of every voxel (TestFrame.cv)
    int tcv = 0;                         //   and the offset tables of its bricks (int32 d1 + d2 + d3)
    int64_t tcv_bytes = 0;
    vr::DevBuf tcol;                     // TEST axis views: per corner line a mask of occupied cells along
    int tca[3] = {1, 1, 1}, tnca[3] = {0, 0, 0};   // the axis (tca voxels per cell, tnca <= 64 cells),
    int64_t tcol_base[3] = {0, 0, 0};    //   the three axes' tables back to back
    int tcol_pitch[3] = {0, 0, 0};
    bool idx64 = false;
    // class-volume brick layout (bx, by, bz voxels per brick, bricks x-major); 1x1x1 = the linear
    // x-major layout of the reference.  offset(x,y,z) = Fx[x] + Fy[y] + Fz[z] (separable).
    int brick[3] = {4, 4, 8};
    int64_t cls_bytes = 0;               // bytes of cls_vrc (packed at cbits < 8)
    int64_t cls_slots = 0;               // class slots (voxels and brick padding) of the layout
    int cbits = 8;                       // bits per class in cls_vrc: 2, 4 or 8 (build_layout)
    vr::DevBuf cls8;                     // cbits < 8: the classes one byte per slot (occupancy pass)
    std::vector<int64_t> lay;            // Fx (d1) | Fy (d2) | Fz (d3)
    // general views of a compact (cbits < 8), 32-bit volume march a byte-per-class copy in the
    // options' brick (plain byte gathers: no bit extraction, fewer VGPRs); axis-aligned views keep
    // the compact volume.  gen = the copy exists (else every view marches cls_vrc).
    bool gen = false;
    bool leafcols = false;   // occ_leafcols holds the axis views' leaf-column masks (vr_options.leaf_columns)
    vr::DevBuf cls_gen, layout_gen, pmaps_gen;
    vr::DevBuf pmaps_pad, pmaps_gen_pad;   // general 32-bit views: the maps with kMapPadMax kMapOut either side
    std::vector<int64_t> lay_gen;
    int64_t gen_bytes = 0;
    int batch = 0;                       // samples per straight-line batch per lane (0: auto, 8 or 16)
    int occ_lds = 1;
    int axis1_ok = 1;                    // use the axis-aligned specialisation when it applies
    int persist_wgs = 0;                 // persistent launch (workgroups per CU), 0 = one per work tile
    int order_mode = 0;                  // work-tile order (see work_for)
    int cull = 2;                        // whole-frame renders skip the tiles off the projected box (1: its
                                         // bounding rectangle; 2: and, in the march, the work tiles off its hull)
    int tab_reuse = 1;                   // AXIS1 view table: reuse the copy the last launch of this view published
    int test_axz = 1;                    // TEST axis views march plane by plane (test_axis_kernel)
    vr_options opt;                      // the options the context was created with / last set
    struct AxTab {
        vr::DevBuf buf;                      // the published copy
        std::vector<uint32_t> key;       // the view it belongs to (empty: none published)
    };
    std::map<hipStream_t, AxTab> axtab;  // one per stream: launches are ordered on their own stream only
    struct FrameList {
        vr::WorkCache wc;                // the device-built whole-frame work list
        std::vector<uint32_t> key;       // W, H, the visible rectangle and the column cull it was built for
    };
    std::map<hipStream_t, FrameList> frame_lists;   // per stream, like axtab
    struct ZTab {                        // TEST axis views: the march axis's per-frame tables (LDS image)
        vr::DevBuf buf;
        std::vector<uint32_t> key;       // the inputs they were built from
        std::vector<int32_t> host;       // (kept: the upload may still read it)
        int words = 0;
    };
    std::map<hipStream_t, ZTab> ztabs;   // per stream, like axtab
    int occ_lo[3] = {0, 0, 0}, occ_hi[3] = {-1, -1, -1};   // occupied macro-cell range per axis
    // per axis a: summed-area table over the (a0, a1) plane (the other two axes, ascending) of the
    // cell columns along a holding an occupied cell, (ncell + 1)^2 entries (farm-tile cull of
    // axis-parallel views, vr_api.cpp visible_tiles)
    std::vector<int32_t> col_sat[3];
    vr::DevBuf col_sat_dev;              // the three column tables on the device (worklist_kernel's cull)
    uint32_t sat_gen = 0;                // bumped whenever they change (frame-list keys)
    // super cells (2^sc_shift macro cells per axis, <= 16 per axis): occupied flags, x-major; the
    // farm-tile cull of general orthographic views projects the occupied ones (visible_tiles)
    int sc_shift = 0, nsc = 0;
    std::vector<uint8_t> socc;
    // visible_tiles results by (camera, params, tile size, cull): a steady view is planned once
    // (cleared when the classes change)
    mutable std::map<std::vector<uint32_t>, std::vector<int32_t>> vis_cache;
    bool cls_test_valid = false;
    // TEST: a voxel on the volume's faces is not class 0 (test_faces_kernel; 1 until classified)
    vr::DevBuf faces_flag;
    int32_t test_faces_dirty = 1;
    int ncell = 0, cb_shift = 0;
    std::vector<vr_tf_interval> tf;
    int cls0_vrc = 0, cls0_test = 0;
    bool zero_transparent = true;
    std::map<std::tuple<int, int, int, int, int, int, std::vector<int32_t>>, std::unique_ptr<vr::WorkCache>> work_cache;
    std::map<std::tuple<int, int, int, int, int, int, std::vector<int32_t>>, std::unique_ptr<vr::DevBuf>> slot_maps;
    unsigned long long* count_ptr = nullptr;   // vr_count_marched: launch_frame runs the counting march
    bool timing = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_free, ev_pending;
    double timing_ms = 0;
    int64_t timing_launches = 0;
    vr::Group* group = nullptr;          // multi-GPU context: the other devices' parts + RCCL (vr_multi.cpp)
    vr::Group* part_of = nullptr;        // the group this context is a part of (every part, the first too):
                                         // its host waits are polled against the group's deadline
    std::vector<vr::Retired> retired;    // evicted cache buffers waiting for their readers (retire_buffers)
    hipEvent_t switch_ev = nullptr;      // vr_set_stream: the new stream is ordered after the old one
};


namespace vr {

// shared internals (vr_api.cpp)
// d1 * d2 * d3 for a volume: every dim positive (VR_EINVAL) and the float32 byte count within
// size_t / int64 (VR_ERANGE), checked before anything is allocated
size_t checked_count(int64_t d1, int64_t d2, int64_t d3);
void set_device(vr_ctx* c);
void check_params(const vr_params* p);
vr_ctx* create_common(const float* voxels, bool on_device, int64_t d1, int64_t d2, int64_t d3, double cal_max,
                      const vr_tf_interval* tf, int32_t n_tf, int32_t device, const vr_options* opt_in,
                      DevBuf* adopt_vol = nullptr);
std::vector<int32_t> visible_tiles(const vr_ctx* c, const vr_params* p, const vr_camera* cam, int tw, int th);
// renders the listed user tiles (tile_w x tile_h, x-major ids) into the compact buffer d_tiles on c->stream
void render_tile_list(vr_ctx* c, const vr_params* p, const vr_camera* cam, int tile_w, int tile_h,
                      const std::vector<int32_t>& list, float* d_tiles, int out_rgb);
// scatter: tile tiles[i] from block slots[i] of d_tiles; every other pixel = background (one frame)
void assemble_slots(vr_ctx* c, int W, int H, int tile_w, int tile_h, const std::vector<int32_t>& tiles,
                    const std::vector<int32_t>& slots, int n_blocks, const float* d_tiles, const float background[4],
                    float* d_frame, int out_rgb);
void destroy_ctx_single(vr_ctx* c);
// Moves the buffers into c->retired behind events on the context's streams (its stream, and the
// auxiliary one of frames in flight: between batches the auxiliary stream is joined into the ctx
// stream, and vr_set_stream orders a new stream after the old one, so these cover every launch),
// freeing earlier batches whose events have completed.
void retire_buffers(vr_ctx* c, const std::vector<DevBuf*>& bufs, std::vector<std::vector<int32_t>>* hosts = nullptr);
void reap_retired(vr_ctx* c, bool wait);
// collects the finished per-launch timing events of c (synchronises c->stream)
void drain_timing(vr_ctx* c);
// Frames in flight: launch(f) for f < n with c->stream set to the ctx stream (even f) or the
// auxiliary stream (odd f), both forked from and joined back into the ctx stream.
void frames_in_flight(vr_ctx* c, int n, const std::function<void(int)>& launch);
WorkCache* work_for_subset(vr_ctx* c, int W, int H, int tile, const std::vector<int32_t>& own,
                           const std::vector<int32_t>& visible);
void launch_frame(vr_ctx* c, const vr_params* p, const vr_camera* cam, WorkCache* wc, float4* out, int out_tiles,
                  int tile_w, int tile_h, int out_rgb = 0);
void launch_frame(vr_ctx* c, const vr_params* p, const vr_camera* cam, const WorkView& wv, float4* out, int out_tiles,
                  int tile_w, int tile_h, int out_rgb = 0);
// the multi-GPU plan kernel (vr_kernels.hip plan_kernel): per frame of a batch, this part's work list
// and (rank 0) the scatter map of the peers' tiles, from the frame's tile owners
hipError_t launch_plan(const int8_t* owner, int n_frames, int ntiles, int nty, int W, int H, int tile, int rank,
                       int n_ranks, const int32_t* woff, const int32_t* nown, const int32_t* mbase, WorkTile* work,
                       int32_t* map, hipStream_t st);
hipError_t launch_scatter_tiles(int W, int H, int tile, const int32_t* map, int n_tiles, const float* tiles,
                                float4* frames, hipStream_t st);

// multi-GPU (vr_multi.cpp)
void group_render(vr_ctx* c, const vr_params* p, const vr_camera* cams, int n, float* out, int32_t out_flags);
void group_destroy(Group* g);
void group_for_each(vr_ctx* c, void (*fn)(vr_ctx*, void*), void* arg);   // every device part, c first
void group_options_changed(vr_ctx* c);
void group_sync(vr_ctx* c);   // every part's stream and comm stream
// Host wait for stream s of context c: hipStreamSynchronize, or -- for a part of a multi-GPU
// context -- the group's polled wait (RCCL errors and comm_timeout_ms abort the group, VR_ECOMM)
void ctx_sync(vr_ctx* c, hipStream_t s);
// VR_ECOMM if c is a part of a multi-GPU context that has failed
void group_check_alive(vr_ctx* c);
// progress marker on c->stream (parts of multi-GPU contexts; a no-op otherwise): the group's host
// waits restart their comm_timeout_ms deadline whenever one completes
void group_mark(vr_ctx* c);
void group_mark_stream(Group* g, int device, hipStream_t s);

}  // namespace vr
