// vr_multi.cpp -- multi-GPU contexts behind the C-ABI: the screen is cut into
// tile x tile tiles, the tiles that can hold a non-background pixel (vr_visible_tiles) are dealt to
// the GPUs interleaved, every GPU marches its tiles into a compact RGB buffer, and the buffers are
// gathered into the first GPU over xGMI, where one assembly launch writes the [x*H + y] frame (the
// exact background everywhere else).  The volume is RCCL-broadcast from the first GPU once, at
// creation; every GPU then builds its own classes, occupancy and tables.
//
// The reference renders on one GPU only (cudaSetDevice(0), kernel.cu:885, myApp.cu:818); rays are
// independent (blendSampleColors reads only its own samples, kernel.cu:205-209), so a farmed frame
// equals the one-GPU frame bit for bit.
//
// Two ways to hold a group:
//   vr_create_multi -- one process drives n GPUs (ncclCommInitAll over the device list).  A device
//                      list that repeats a GPU (a rehearsal of the plan on fewer GPUs: RCCL refuses
//                      two ranks on one device) moves the tiles with hipMemcpyPeerAsync instead.
//   vr_create_rank  -- one process per GPU (torchrun / MPI style): ncclCommInitRank with an id from
//                      vr_comm_unique_id that the caller distributes; every rank calls vr_render with
//                      the same params and camera, rank 0 receives the frame.
// Per frame, rank r's tiles travel with ncclSend on its own stream and rank 0 posts one ncclRecv per
// peer inside one ncclGroupStart/End, so each peer uses its own xGMI link into rank 0 (NCCL has no
// gather primitive; a ring would be bound by one link).
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <deque>
#include <thread>

#include "ctx.h"

#pragma clang fp contract(off)

namespace vr {

namespace {

inline void nccl_check(ncclResult_t r, const char* what) {
    if (r != ncclSuccess) {
        g_last_hip_error = std::string(what) + ": " + ncclGetErrorString(r);
        throw Error(VR_ECOMM, g_last_hip_error.c_str());
    }
}

}  // namespace

struct Group {
    // Failure detection (SURVEY 5 failure row): every host wait on a part's stream is a poll of the
    // stream and of the communicators' asynchronous errors against a deadline (comm_timeout_ms).  An
    // RCCL error, a HIP error or the deadline aborts every communicator of the group (ncclCommAbort
    // releases peers blocked in a send / receive) and fails the call with VR_ECOMM; later calls fail
    // the same way until the context is destroyed.
    int timeout_ms = 60000;               // 0: wait forever
    std::string failed;                   // non-empty: the group has failed (the reason)
    int n_ranks = 1;                      // ranks of the group (GPUs)
    int rank0 = 0;                        // global rank of parts[0] (multi-process: this process's rank)
    std::vector<vr_ctx*> parts;           // parts[0] = the owning context (not owned here), others owned
    std::vector<ncclComm_t> comms;        // one per part; empty for the peer-copy transport / one rank
    bool peer_copy = false;               // single process over repeated devices: hipMemcpyPeerAsync
    int tile = 64;
    float w0 = 1.0f;                      // rank 0's weight in the tile deal (others 1)
    // Transfers run on a comm stream per part, double-buffered (k = frame & 1), so frame f's
    // transfer overlaps frame f + 1's march.  Events order the buffers' reuse.
    std::vector<hipStream_t> cs;          // per part: comm stream (on the part's GPU)
    std::vector<DevBuf> send[2];          // peers: their tiles, compact RGB
    DevBuf recv[2];                       // rank 0: the peers' tiles, rank-major blocks
    std::vector<hipEvent_t> ready;        // per part: its march of the current frame done (its stream)
    std::vector<hipEvent_t> sent[2];      // per part: buffer k's transfer done (comm stream of the copy)
    std::vector<bool> sent_pending[2];
    hipEvent_t recvd[2] = {nullptr, nullptr};       // rank 0: buffer k received (cs[0])
    hipEvent_t scattered[2] = {nullptr, nullptr};   // rank 0: buffer k scattered into the frame
    bool scattered_pending[2] = {false, false};
    uint64_t frame_no = 0;
    // Peer traffic (vr_group_traffic_read): per part, the tile bytes it posted to rank 0 (send) and,
    // on rank 0, the bytes it posted to receive; frames rendered by the group.  Since the last reset.
    std::vector<int64_t> tx_bytes, rx_bytes, tx_frames;   // (per part: a reset clears that part's only)
    // plans: one per distinct visible-tile list (a pure function of the camera), cached
    struct Plan {
        std::vector<int32_t> ids;                   // visible tiles, ascending
        std::vector<std::vector<int32_t>> lists;    // per global rank
    };
    int W = -1, H = -1;                   // frame size the cached plans are for
    std::map<std::vector<int32_t>, Plan> plans;
    const Plan* last = nullptr;           // the last frame's plan (vr_group_tiles)
    // Device-side plans (plan_kernel): per batch the host uploads only the frames' tile owners and a
    // few offsets (asynchronously, from a pinned staging ring), and every part expands them into its
    // work lists (rank 0 also the scatter map) on its own stream.
    struct PartPlan {
        DevBuf blob;   // owners | per-part work offsets | rank 0's own-entry counts | map bases
        DevBuf work;   // this part's work lists of the batch, frame after frame
        DevBuf map;    // rank 0: (tile, frame) per receive block
    };
    std::vector<PartPlan> pp;
    struct Stage {     // pinned host copy of a batch's blob; reusable once every part's copy is done
        void* h = nullptr;
        size_t bytes = 0;
        std::vector<hipEvent_t> ev;   // per part, on its stream after its copy
        std::vector<bool> pend;
    };
    std::vector<Stage> stage;
    size_t stage_next = 0;
    // Progress markers: an event recorded after every frame a part marches, every classification
    // step and every broadcast piece.  A host wait's deadline counts from the last marker seen
    // complete (or from the wait's start): comm_timeout_ms bounds a lack of progress, not the length
    // of legitimately queued work (a long batch, a C5-size classification or broadcast).
    struct Marker {
        int device;
        hipEvent_t ev;
    };
    std::deque<Marker> markers;           // recorded, not yet seen complete
    std::vector<Marker> marker_pool;      // seen complete: reusable
};

namespace {
constexpr size_t kMaxMarkers = 512;   // pending markers; beyond that no new ones (the old still report)

// Pending markers that have completed go back to the pool; true if any did (progress).
bool markers_progress(Group* g) {
    bool any = false;
    for (auto it = g->markers.begin(); it != g->markers.end();) {
        if (hipEventQuery(it->ev) == hipErrorNotReady) { ++it; continue; }
        g->marker_pool.push_back(*it);   // (an error also ends the marker: the stream wait reports it)
        it = g->markers.erase(it);
        any = true;
    }
    return any;
}
}  // namespace

void group_mark_stream(Group* g, int device, hipStream_t s) {
    if (!g || g->timeout_ms <= 0 || !g->failed.empty()) return;
    if (g->markers.size() >= kMaxMarkers) {
        markers_progress(g);
        if (g->markers.size() >= kMaxMarkers) return;
    }
    Group::Marker m{device, nullptr};
    for (size_t i = 0; i < g->marker_pool.size(); ++i)
        if (g->marker_pool[i].device == device) {
            m = g->marker_pool[i];
            g->marker_pool.erase(g->marker_pool.begin() + (std::ptrdiff_t)i);
            break;
        }
    if (!m.ev) hip_check(hipEventCreateWithFlags(&m.ev, hipEventDisableTiming));   // (device is current)
    hip_check(hipEventRecord(m.ev, s));
    g->markers.push_back(m);
}

void group_mark(vr_ctx* c) {
    if (c->part_of) group_mark_stream(c->part_of, c->device, c->stream);
}

namespace {

// Deals the ids to n ranks, rank 0 with weight w0 and every other rank weight 1, interleaved: tile i
// goes to the rank furthest below its target share of the first i + 1 tiles (ties: lowest rank).
// Deterministic, so every rank derives the same plan (volumerenderingproject_amd/distributed.py
// weighted_lists states the same deal).
std::vector<std::vector<int32_t>> weighted_lists(const std::vector<int32_t>& ids, int n, double w0) {
    std::vector<std::vector<int32_t>> lists((size_t)n);
    const double tot = w0 + (n - 1);
    for (size_t i = 0; i < ids.size(); ++i) {
        int best = 0;
        double bd = 0;
        for (int r = 0; r < n; ++r) {
            const double d = (r == 0 ? w0 : 1.0) / tot * (double)(i + 1) - (double)lists[(size_t)r].size();
            if (r == 0 || d > bd + 1e-12) { best = r; bd = d; }
        }
        lists[(size_t)best].push_back(ids[i]);
    }
    return lists;
}

// (the cache is trimmed only by group_render before a batch collects its plans: the batch holds
// pointers into it)
const Group::Plan& plan_for(Group* g, std::vector<int32_t>&& ids) {
    auto it = g->plans.find(ids);
    if (it == g->plans.end()) {
        Group::Plan pl;
        pl.ids = ids;
        pl.lists = weighted_lists(pl.ids, g->n_ranks, g->w0);
        it = g->plans.emplace(std::move(ids), std::move(pl)).first;
    }
    return it->second;
}

void abort_comms(std::vector<ncclComm_t>& comms) {
    for (ncclComm_t& cm : comms)
        if (cm) {
            (void)ncclCommAbort(cm);   // (also frees it: an aborted communicator is not destroyed again)
            cm = nullptr;
        }
}

[[noreturn]] void group_fail(Group* g, const std::string& why) {
    abort_comms(g->comms);
    if (g->failed.empty()) g->failed = why;
    g_last_hip_error = why;
    throw Error(VR_ECOMM, why);
}

// Waits until `done()` holds, polling: the communicators' asynchronous errors and the deadline are
// checked between polls.  On an RCCL error or when the deadline passes, every communicator in
// `comms` is aborted and the wait throws VR_ECOMM with the reason (`fail`).  The deadline restarts
// whenever `progress()` reports that queued work has moved on (a group's markers completing).
template <class Done, class Fail, class Progress>
void poll_until(Done&& done, const std::vector<ncclComm_t>& comms, int timeout_ms, const char* what, Fail&& fail,
                Progress&& progress) {
    auto t0 = std::chrono::steady_clock::now();
    for (unsigned it = 0;; ++it) {
        if (done()) return;
        if (progress()) t0 = std::chrono::steady_clock::now();
        for (ncclComm_t cm : comms) {
            if (!cm) continue;
            ncclResult_t r = ncclSuccess;
            if (ncclCommGetAsyncError(cm, &r) == ncclSuccess && r != ncclSuccess && r != ncclInProgress)
                fail(std::string("RCCL error while waiting for ") + what + ": " + ncclGetErrorString(r));
        }
        if (timeout_ms > 0) {
            const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            if (ms > (double)timeout_ms)
                fail(std::string("timed out after ") + std::to_string(timeout_ms) + " ms waiting for " + what +
                     " (communicators aborted)");
        }
        if (it < 256) std::this_thread::yield();
        else std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}

// One stream of the group drained (polled, with the group's deadline).  A HIP error on it also
// aborts the group: the other ranks would otherwise wait forever for this part's tiles.
void wait_stream(Group* g, hipStream_t s, const char* what) {
    if (!g->failed.empty()) throw Error(VR_ECOMM, "multi-GPU context failed earlier: " + g->failed);
    poll_until(
        [&] {
            const hipError_t q = hipStreamQuery(s);
            if (q == hipErrorNotReady) return false;
            if (q != hipSuccess) group_fail(g, std::string("HIP error on ") + what + ": " + hipGetErrorString(q));
            return true;
        },
        g->comms, g->timeout_ms, what, [&](const std::string& why) { group_fail(g, why); },
        [&] { return markers_progress(g); });
}

void wait_event(Group* g, hipEvent_t e, const char* what) {
    if (!g->failed.empty()) throw Error(VR_ECOMM, "multi-GPU context failed earlier: " + g->failed);
    poll_until(
        [&] {
            const hipError_t q = hipEventQuery(e);
            if (q == hipErrorNotReady) return false;
            if (q != hipSuccess) group_fail(g, std::string("HIP error on ") + what + ": " + hipGetErrorString(q));
            return true;
        },
        g->comms, g->timeout_ms, what, [&](const std::string& why) { group_fail(g, why); },
        [&] { return markers_progress(g); });
}

void sync_all(Group* g) {
    for (size_t i = 0; i < g->parts.size(); ++i) {
        vr_ctx* pc = g->parts[i];
        set_device(pc);
        wait_stream(g, pc->stream, "a part's render stream");
        if (i < g->cs.size() && g->cs[i]) wait_stream(g, g->cs[i], "a part's RCCL stream");
    }
}

hipEvent_t new_event() {
    hipEvent_t e;
    hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    return e;
}

constexpr size_t kStageSlots = 4;      // staging slots created with the group
constexpr size_t kStageSlotsMax = 64;  // batches whose blob uploads may be in flight before the host waits

// comm streams and events, created on first use (per part, on its GPU)
void ensure_comm(Group* g) {
    const size_t n = g->parts.size();
    if (g->cs.size() == n) return;
    g->cs.assign(n, nullptr);
    g->ready.assign(n, nullptr);
    for (int k = 0; k < 2; ++k) {
        g->send[k] = std::vector<DevBuf>(n);
        g->sent[k].assign(n, nullptr);
        g->sent_pending[k].assign(n, false);
    }
    for (size_t i = 0; i < n; ++i) {
        set_device(g->parts[i]);
        hip_check(hipStreamCreateWithFlags(&g->cs[i], hipStreamNonBlocking));
        g->ready[i] = new_event();
        for (int k = 0; k < 2; ++k) g->sent[k][i] = new_event();
    }
    set_device(g->parts[0]);
    for (int k = 0; k < 2; ++k) {
        g->recvd[k] = new_event();
        g->scattered[k] = new_event();
    }
    g->pp = std::vector<Group::PartPlan>(n);
    g->stage = std::vector<Group::Stage>(kStageSlots);
    for (Group::Stage& s : g->stage) {
        s.ev.assign(n, nullptr);
        s.pend.assign(n, false);
        for (size_t i = 0; i < n; ++i) {
            set_device(g->parts[i]);
            s.ev[i] = new_event();
        }
    }
}

Group* new_group(vr_ctx* c, int n_ranks, int rank0) {
    Group* g = new Group;
    g->n_ranks = n_ranks;
    g->rank0 = rank0;
    g->w0 = c->opt.farm_rank0_weight;
    g->tile = c->opt.farm_tile;
    g->timeout_ms = c->opt.comm_timeout_ms;
    g->parts.push_back(c);
    c->part_of = g;
    return g;
}

// Broadcast of the first part's volume into bufs[i] (i >= 1, on parts' devices) over the group's
// communicators, in 1 GiB pieces (bounded messages for the 34.4 GB C5 replica).
void broadcast_volume(Group* g, vr_ctx* root, const std::vector<int>& devices, std::vector<DevBuf>& bufs,
                      size_t count) {
    const size_t chunk = (size_t)1 << 28;
    std::vector<hipStream_t> st(devices.size());
    for (size_t i = 0; i < devices.size(); ++i) {
        hip_check(hipSetDevice(devices[i]));
        hip_check(hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking));
    }
    hip_check(hipSetDevice(devices[0]));
    wait_stream(g, root->stream, "the volume upload");   // the root's volume copy has landed
    for (size_t o = 0; o < count; o += chunk) {
        const size_t n = std::min(chunk, count - o);
        if (g->peer_copy) {
            for (size_t i = 1; i < devices.size(); ++i)
                hip_check(hipMemcpyPeerAsync(bufs[i].as<float>() + o, devices[i], root->vol.as<float>() + o,
                                             devices[0], n * sizeof(float), st[0]));
        } else {
            nccl_check(ncclGroupStart(), "ncclGroupStart");
            for (size_t i = 0; i < devices.size(); ++i) {
                float* p = i == 0 ? root->vol.as<float>() + o : bufs[i].as<float>() + o;
                nccl_check(ncclBroadcast(p, p, n, ncclFloat32, 0, g->comms[i], st[i]), "ncclBroadcast (volume)");
            }
            nccl_check(ncclGroupEnd(), "ncclGroupEnd");
        }
        hip_check(hipSetDevice(devices[0]));
        group_mark_stream(g, devices[0], st[0]);   // (progress: one marker per piece)
    }
    try {
        for (size_t i = 0; i < devices.size(); ++i) {
            hip_check(hipSetDevice(devices[i]));
            wait_stream(g, st[i], "the volume broadcast");
        }
    } catch (...) {   // (after an abort the streams drain: RCCL's kernels see the abort flag)
        for (size_t i = 0; i < devices.size(); ++i) {
            (void)hipSetDevice(devices[i]);
            (void)hipStreamSynchronize(st[i]);
            (void)hipStreamDestroy(st[i]);
        }
        throw;
    }
    for (size_t i = 0; i < devices.size(); ++i) {
        hip_check(hipSetDevice(devices[i]));
        hip_check(hipStreamDestroy(st[i]));
    }
}

// vr_create_rank before its group exists: a polled wait on `st` with the options' deadline; on
// failure the communicator is aborted (and nulled) and VR_ECOMM thrown
void rank_wait(hipStream_t st, ncclComm_t& comm, const vr_options* options, const char* what) {
    vr_options o;
    vr_options_default(&o);
    if (options) o = *options;
    std::vector<ncclComm_t> comms{comm};
    auto fail = [&](const std::string& why) {
        abort_comms(comms);
        comm = nullptr;
        g_last_hip_error = why;
        throw Error(VR_ECOMM, why);
    };
    poll_until(
        [&] {
            const hipError_t q = hipStreamQuery(st);
            if (q == hipErrorNotReady) return false;
            if (q != hipSuccess) fail(std::string("HIP error during ") + what + ": " + hipGetErrorString(q));
            return true;
        },
        comms, o.comm_timeout_ms, what, fail, [] { return false; });   // (one collective: no markers)
}

}  // namespace

void group_destroy(Group* g) {
    if (!g) return;
    try {
        if (!g->failed.empty()) throw 0;
        sync_all(g);
    } catch (...) {
        // a failed group (communicators aborted, so RCCL's kernels have exited) may still have
        // marches queued: drain every stream before anything is freed under them
        for (size_t i = 0; i < g->parts.size(); ++i) {
            (void)hipSetDevice(g->parts[i]->device);
            (void)hipStreamSynchronize(g->parts[i]->stream);
            if (i < g->cs.size() && g->cs[i]) (void)hipStreamSynchronize(g->cs[i]);
        }
    }
    for (size_t i = 0; i < g->cs.size(); ++i) {
        (void)hipSetDevice(g->parts[i]->device);
        (void)hipEventDestroy(g->ready[i]);
        for (int k = 0; k < 2; ++k) {
            (void)hipEventDestroy(g->sent[k][i]);
            g->send[k][i].reset();
        }
        (void)hipStreamDestroy(g->cs[i]);
    }
    (void)hipSetDevice(g->parts[0]->device);
    for (int k = 0; k < 2; ++k) {
        if (g->recvd[k]) (void)hipEventDestroy(g->recvd[k]);
        if (g->scattered[k]) (void)hipEventDestroy(g->scattered[k]);
        g->recv[k].reset();
    }
    for (size_t i = 0; i < g->pp.size() && i < g->parts.size(); ++i) {
        (void)hipSetDevice(g->parts[i]->device);
        g->pp[i].blob.reset();
        g->pp[i].work.reset();
        g->pp[i].map.reset();
    }
    for (Group::Stage& s : g->stage) {
        for (size_t i = 0; i < s.ev.size(); ++i)
            if (s.ev[i]) {
                (void)hipSetDevice(g->parts[i]->device);
                (void)hipEventDestroy(s.ev[i]);
            }
        if (s.h) (void)hipHostFree(s.h);
    }
    for (const Group::Marker& m : g->markers) {   // (the streams are drained above)
        (void)hipSetDevice(m.device);
        (void)hipEventDestroy(m.ev);
    }
    for (const Group::Marker& m : g->marker_pool) {
        (void)hipSetDevice(m.device);
        (void)hipEventDestroy(m.ev);
    }
    for (ncclComm_t cm : g->comms)
        if (cm) (void)ncclCommDestroy(cm);
    for (vr_ctx* pc : g->parts) pc->part_of = nullptr;
    for (size_t i = 1; i < g->parts.size(); ++i) destroy_ctx_single(g->parts[i]);
    delete g;
}

void group_options_changed(vr_ctx* c) {
    Group* g = c->group;
    if (!g) return;
    sync_all(g);
    g->timeout_ms = c->opt.comm_timeout_ms;
    g->w0 = c->opt.farm_rank0_weight;
    g->tile = c->opt.farm_tile;
    g->plans.clear();   // re-plan at the next frame
    g->last = nullptr;
    g->W = g->H = -1;
}

void group_for_each(vr_ctx* c, void (*fn)(vr_ctx*, void*), void* arg) {
    if (!c->group) {
        fn(c, arg);
        return;
    }
    for (vr_ctx* pc : c->group->parts) fn(pc, arg);
}

void group_sync(vr_ctx* c) {
    if (c->group) sync_all(c->group);
}

void group_check_alive(vr_ctx* c) {
    if (c->part_of && !c->part_of->failed.empty())
        throw Error(VR_ECOMM, "multi-GPU context failed earlier: " + c->part_of->failed);
}

void ctx_sync(vr_ctx* c, hipStream_t s) {
    if (c->part_of) wait_stream(c->part_of, s, "a part's stream");
    else hip_check(hipStreamSynchronize(s));
}

// Work tiles (16 x 16 rays) of user tile t of a tile x tile grid that lie inside the W x H frame
inline int tile_work_tiles(int t, int nty, int W, int H, int tile) {
    const int tx = t / nty, ty = t % nty, per = tile / kWgRaysX;
    const int nx = std::min(per, (W - tx * tile + kWgRaysX - 1) / kWgRaysX);
    const int ny = std::min(per, (H - ty * tile + kWgRaysY - 1) / kWgRaysY);
    return nx * ny;
}

// A batch of n frames, frame f rendered with cams[f] into out + f*W*H*4: every part marches each
// frame's tiles (rank 0 straight into the frame), the batch's peer tiles travel in ONE RCCL group
// (one ncclSend per peer, one ncclRecv per peer on rank 0: the host cost of a collective is paid
// once per batch) and ONE scatter launch writes them into their frames.
//
// Planning: the host derives each frame's visible tiles and their deal (both pure functions of the
// camera, cached per view), i.e. the tile owners and the per-rank counts that size the transfers.
// It uploads only the owners and a few offsets per batch, asynchronously from a pinned staging ring;
// every part's plan_kernel expands them on its own stream into its work lists (and on rank 0 the
// scatter map).  No host synchronisation per frame: a moving camera costs the host its planning
// arithmetic and the launches.
void group_render(vr_ctx* c, const vr_params* p, const vr_camera* cams, int n, float* out, int32_t out_flags) {
    Group* g = c->group;
    const int T = g->tile, W = p->width, H = p->height;
    const bool holds_rank0 = g->rank0 == 0;
    const bool out_on_device = (out_flags & VR_OUT_DEVICE) != 0;
    if (n <= 0) throw Error(VR_EINVAL, "vr_render_batch: n_frames must be positive");
    if (!g->failed.empty()) throw Error(VR_ECOMM, "multi-GPU context failed earlier: " + g->failed);
    if (holds_rank0 && !out) throw Error(VR_EINVAL, "vr_render: rank 0 of a multi-GPU context needs an output");
    // the plans: every rank derives the same visible-tile list from the same camera (no exchange)
    std::vector<const Group::Plan*> pl((size_t)n);
    if (W != g->W || H != g->H || g->plans.size() + (size_t)n > 64) {   // no plan pointer is held here
        g->plans.clear();
        g->last = nullptr;
        g->W = W; g->H = H;
    }
    for (int f = 0; f < n; ++f) pl[(size_t)f] = &plan_for(g, visible_tiles(c, p, &cams[f], T, T));
    g->last = pl[(size_t)n - 1];
    ensure_comm(g);
    const size_t per = (size_t)T * T * 3;   // floats per RGB tile (alpha is 1 by construction)
    const size_t fpx = (size_t)W * H * 4;   // floats per frame
    const int n_parts = (int)g->parts.size();
    const int N = g->n_ranks;
    const int k = (int)(g->frame_no++ & 1);
    const int ntx = (W + T - 1) / T, nty = (H + T - 1) / T, ntiles = ntx * nty;
    // ---- host side of the plan: owners, counts, offsets ----
    // cnt[q][f] tiles of rank q in frame f; wt[q][f] their work tiles; bg[f] work tiles of the
    // invisible tiles (rank 0 stores their background)
    std::vector<int32_t> cnt((size_t)N * n), wt((size_t)N * n), bgwt((size_t)n);
    const size_t own_bytes = ((size_t)n * ntiles + 15) / 16 * 16;
    // blob: owners (int8, n x ntiles) | woff (n_parts x n) | nown (n) | mbase (n x N), int32 after the owners
    const size_t n_i32 = (size_t)n_parts * n + n + (size_t)n * N;
    const size_t blob_bytes = own_bytes + n_i32 * sizeof(int32_t);
    // a staging slot whose previous blob every part has copied; the ring grows (up to
    // kStageSlotsMax) rather than wait while the GPUs are behind, so queuing batches ahead of a busy
    // GPU never blocks the host (only a ring of kStageSlotsMax batches in flight does)
    auto slot_free = [&](Group::Stage& s) {
        for (int i = 0; i < n_parts; ++i)
            if (s.pend[(size_t)i]) {
                set_device(g->parts[(size_t)i]);
                const hipError_t q = hipEventQuery(s.ev[(size_t)i]);
                if (q == hipErrorNotReady) return false;
                hip_check(q);
                s.pend[(size_t)i] = false;
            }
        return true;
    };
    size_t si = g->stage.size();
    for (size_t j = 0; j < g->stage.size() && si == g->stage.size(); ++j) {
        const size_t c2 = (g->stage_next + j) % g->stage.size();
        if (slot_free(g->stage[c2])) si = c2;
    }
    if (si == g->stage.size() && g->stage.size() < kStageSlotsMax) {
        Group::Stage s;
        s.ev.assign((size_t)n_parts, nullptr);
        s.pend.assign((size_t)n_parts, false);
        for (int i = 0; i < n_parts; ++i) {
            set_device(g->parts[(size_t)i]);
            s.ev[(size_t)i] = new_event();
        }
        g->stage.push_back(std::move(s));
        si = g->stage.size() - 1;
    }
    if (si == g->stage.size()) {   // kStageSlotsMax batches in flight: wait for the oldest slot
        si = g->stage_next % g->stage.size();
        for (int i = 0; i < n_parts; ++i)
            if (g->stage[si].pend[(size_t)i]) {
                set_device(g->parts[(size_t)i]);
                wait_event(g, g->stage[si].ev[(size_t)i], "a staging upload");
                g->stage[si].pend[(size_t)i] = false;
            }
    }
    g->stage_next = si + 1;
    Group::Stage& st = g->stage[si];
    if (st.bytes < blob_bytes) {
        if (st.h) hip_check(hipHostFree(st.h));
        st.h = nullptr;
        st.bytes = 0;
        set_device(c);
        hip_check(hipHostMalloc(&st.h, blob_bytes + 4096, hipHostMallocPortable));
        st.bytes = blob_bytes + 4096;
    }
    int8_t* owner = static_cast<int8_t*>(st.h);
    int32_t* i32 = reinterpret_cast<int32_t*>(static_cast<char*>(st.h) + own_bytes);
    int32_t* woff = i32;                           // [part i][f]
    int32_t* nown = woff + (size_t)n_parts * n;    // [f]
    int32_t* mbase = nown + n;                     // [f][q]
    std::memset(owner, -1, (size_t)n * ntiles);
    int frame_wt = 0;   // work tiles of a whole frame
    for (int t = 0; t < ntiles; ++t) frame_wt += tile_work_tiles(t, nty, W, H, T);
    for (int f = 0; f < n; ++f) {
        const Group::Plan& P = *pl[(size_t)f];
        int vis_wt = 0;
        for (int q = 0; q < N; ++q) {
            int w = 0;
            for (int32_t t : P.lists[(size_t)q]) {
                owner[(size_t)f * ntiles + t] = (int8_t)q;
                w += tile_work_tiles(t, nty, W, H, T);
            }
            cnt[(size_t)q * n + f] = (int32_t)P.lists[(size_t)q].size();
            wt[(size_t)q * n + f] = w;
            vis_wt += w;
        }
        bgwt[(size_t)f] = frame_wt - vis_wt;
        nown[f] = wt[(size_t)f];   // rank 0's own entries come first
    }
    // per peer rank: its tiles of the whole batch (frame-major), and where they land in recv
    std::vector<size_t> cntq((size_t)N, 0), roff((size_t)N + 1, 0);
    for (int q = 1; q < N; ++q)
        for (int f = 0; f < n; ++f) cntq[(size_t)q] += (size_t)cnt[(size_t)q * n + f];
    for (int q = 1; q < N; ++q) roff[(size_t)q + 1] = roff[(size_t)q] + cntq[(size_t)q];
    const size_t n_peer = roff[(size_t)N];
    for (int q = 0; q < N; ++q) {
        size_t b = roff[(size_t)q];
        for (int f = 0; f < n; ++f) {
            mbase[(size_t)f * N + q] = (int32_t)b;
            b += (size_t)cnt[(size_t)q * n + f];
        }
    }
    std::vector<int32_t> entries((size_t)n_parts * n);   // work-list entries of part i, frame f
    std::vector<size_t> total((size_t)n_parts, 0);
    for (int i = 0; i < n_parts; ++i) {
        const int gr = g->rank0 + i;
        int32_t o = 0;
        for (int f = 0; f < n; ++f) {
            const int32_t e = wt[(size_t)gr * n + f] + (gr == 0 ? bgwt[(size_t)f] : 0);
            woff[(size_t)i * n + f] = o;
            entries[(size_t)i * n + f] = e;
            o += e;
        }
        total[(size_t)i] = (size_t)o;
    }
    // ---- every part: upload the blob, expand its plan, march its tiles ----
    float* frames = nullptr;
    if (holds_rank0) {
        set_device(c);
        frames = out;
        if (!out_on_device) {
            c->frame.ensure((size_t)n * fpx * sizeof(float));
            frames = c->frame.as<float>();
        }
    }
    for (int i = 0; i < n_parts; ++i) {
        vr_ctx* pc = g->parts[(size_t)i];
        const int gr = g->rank0 + i;
        Group::PartPlan& pp = g->pp[(size_t)i];
        set_device(pc);
        // (growing a plan buffer retires the old one behind this part's queued work)
        auto grow = [&](DevBuf& b, size_t need) {
            if (need > b.bytes) {
                retire_buffers(pc, {&b});
                b.ensure(need + need / 2);
            }
        };
        grow(pp.blob, blob_bytes);
        grow(pp.work, std::max<size_t>(1, total[(size_t)i]) * sizeof(WorkTile));
        if (gr == 0) grow(pp.map, std::max<size_t>(1, n_peer) * 2 * sizeof(int32_t));
        hip_check(hipMemcpyAsync(pp.blob.p, st.h, blob_bytes, hipMemcpyHostToDevice, pc->stream));
        hip_check(hipEventRecord(st.ev[(size_t)i], pc->stream));
        st.pend[(size_t)i] = true;
        const int32_t* d32 = reinterpret_cast<const int32_t*>(pp.blob.as<char>() + own_bytes);
        hip_check(launch_plan(pp.blob.as<int8_t>(), n, ntiles, nty, W, H, T, gr, N, d32 + (size_t)i * n,
                              d32 + (size_t)n_parts * n, d32 + (size_t)n_parts * n + n, pp.work.as<WorkTile>(),
                              gr == 0 ? pp.map.as<int32_t>() : nullptr, pc->stream));
        auto view = [&](int f) {
            WorkView wv;
            wv.work = pp.work.as<WorkTile>() + woff[(size_t)i * n + f];
            wv.n_work = wv.n_blocks = entries[(size_t)i * n + f];
            wv.bg_first = gr == 0 ? nown[f] : -1;
            return wv;
        };
        if (gr == 0) {
            // rank 0 marches its own tiles straight into each frame (plus the background of every
            // invisible tile); the peers' tiles are scattered in after the gather
            frames_in_flight(pc, n, [&](int f) {
                launch_frame(pc, p, &cams[f], view(f), reinterpret_cast<float4*>(frames + (size_t)f * fpx), 0, 0, 0);
                group_mark(pc);
            });
            continue;
        }
        const size_t mine = cntq[(size_t)gr];
        if (!mine) continue;
        DevBuf& sb = g->send[k][(size_t)i];
        if (mine * per * sizeof(float) > sb.bytes) {   // growing frees the old buffer: drain first
            sync_all(g);
            set_device(pc);
        }
        sb.ensure(mine * per * sizeof(float));
        if (g->sent_pending[k][(size_t)i]) {   // buffer k's previous transfer has read it
            hip_check(hipStreamWaitEvent(pc->stream, g->sent[k][(size_t)i], 0));
            g->sent_pending[k][(size_t)i] = false;
        }
        std::vector<size_t> o((size_t)n + 1, 0);   // each frame's first tile in the send buffer
        for (int f = 0; f < n; ++f) o[(size_t)f + 1] = o[(size_t)f] + (size_t)cnt[(size_t)gr * n + f];
        frames_in_flight(pc, n, [&](int f) {
            launch_frame(pc, p, &cams[f], view(f), reinterpret_cast<float4*>(sb.as<float>() + o[(size_t)f] * per), 1, T,
                         T, 1);
            group_mark(pc);
        });
        hip_check(hipEventRecord(g->ready[(size_t)i], pc->stream));
    }
    // 2. the peers' tiles into rank 0's receive buffer k, on the comm streams
    if (N > 1) {
        if (holds_rank0) {
            set_device(c);
            const size_t need = std::max<size_t>(1, n_peer) * per * sizeof(float);
            if (need > g->recv[k].bytes) {
                sync_all(g);
                set_device(c);
            }
            g->recv[k].ensure(need);
            if (g->scattered_pending[k]) {   // buffer k's previous scatter has read it
                hip_check(hipStreamWaitEvent(g->cs[0], g->scattered[k], 0));
                g->scattered_pending[k] = false;
            }
        }
        if (g->peer_copy) {
            // (every part on one GPU: the copies, their events and rank 0's comm stream share it)
            set_device(c);
            for (int i = 1; i < n_parts; ++i) {
                vr_ctx* pc = g->parts[(size_t)i];
                if (!cntq[(size_t)i]) continue;
                hip_check(hipStreamWaitEvent(g->cs[0], g->ready[(size_t)i], 0));
                hip_check(hipMemcpyPeerAsync(g->recv[k].as<float>() + roff[(size_t)i] * per, c->device,
                                             g->send[k][(size_t)i].as<float>(), pc->device,
                                             cntq[(size_t)i] * per * sizeof(float), g->cs[0]));
                hip_check(hipEventRecord(g->sent[k][(size_t)i], g->cs[0]));
                g->sent_pending[k][(size_t)i] = true;
            }
        } else {
            for (int i = 0; i < n_parts; ++i) {   // comm streams wait for their part's march
                const int gr = g->rank0 + i;
                if (gr == 0 || !cntq[(size_t)gr]) continue;
                set_device(g->parts[(size_t)i]);
                hip_check(hipStreamWaitEvent(g->cs[(size_t)i], g->ready[(size_t)i], 0));
            }
            nccl_check(ncclGroupStart(), "ncclGroupStart");
            for (int i = 0; i < n_parts; ++i) {
                const int gr = g->rank0 + i;
                if (gr != 0) {
                    if (cntq[(size_t)gr])
                        nccl_check(ncclSend(g->send[k][(size_t)i].as<float>(), cntq[(size_t)gr] * per, ncclFloat32, 0,
                                            g->comms[(size_t)i], g->cs[(size_t)i]), "ncclSend (tiles)");
                } else {
                    for (int q = 1; q < N; ++q)
                        if (cntq[(size_t)q])
                            nccl_check(ncclRecv(g->recv[k].as<float>() + roff[(size_t)q] * per, cntq[(size_t)q] * per,
                                                ncclFloat32, q, g->comms[(size_t)i], g->cs[(size_t)i]),
                                       "ncclRecv (tiles)");
                }
            }
            nccl_check(ncclGroupEnd(), "ncclGroupEnd");
            for (int i = 0; i < n_parts; ++i) {
                const int gr = g->rank0 + i;
                if (gr == 0 || !cntq[(size_t)gr]) continue;
                set_device(g->parts[(size_t)i]);
                hip_check(hipEventRecord(g->sent[k][(size_t)i], g->cs[(size_t)i]));
                g->sent_pending[k][(size_t)i] = true;
            }
        }
    }
    // (the traffic the transfers above posted: per part what it sends, rank 0 what it receives)
    if (g->tx_bytes.size() != (size_t)n_parts) {
        g->tx_bytes.assign((size_t)n_parts, 0);
        g->rx_bytes.assign((size_t)n_parts, 0);
        g->tx_frames.assign((size_t)n_parts, 0);
    }
    for (int i = 0; i < n_parts; ++i) {
        const int gr = g->rank0 + i;
        g->tx_frames[(size_t)i] += n;
        if (gr != 0) g->tx_bytes[(size_t)i] += (int64_t)cntq[(size_t)gr] * (int64_t)per * 4;
        else g->rx_bytes[(size_t)i] += (int64_t)n_peer * (int64_t)per * 4;
    }
    // 3. rank 0 scatters the peers' tiles into their frames (its own tiles and the background are
    //    there) through the device-built map
    if (holds_rank0) {
        set_device(c);
        if (n_peer) {
            hip_check(hipEventRecord(g->recvd[k], g->cs[0]));
            hip_check(hipStreamWaitEvent(c->stream, g->recvd[k], 0));
            hip_check(launch_scatter_tiles(W, H, T, g->pp[0].map.as<int32_t>(), (int)n_peer, g->recv[k].as<float>(),
                                           reinterpret_cast<float4*>(frames), c->stream));
            hip_check(hipEventRecord(g->scattered[k], c->stream));
            g->scattered_pending[k] = true;
        }
        if (!out_on_device)
            hip_check(hipMemcpyAsync(out, frames, (size_t)n * fpx * sizeof(float), hipMemcpyDeviceToHost, c->stream));
    }
    if (!out_on_device || !(out_flags & VR_OUT_ASYNC)) sync_all(g);
}

}  // namespace vr

using namespace vr;

extern "C" {

int vr_comm_unique_id(uint8_t id[VR_COMM_ID_BYTES]) {
    if (!id) return VR_EINVAL;
    return guard([&] {
        ncclUniqueId u;
        nccl_check(ncclGetUniqueId(&u), "ncclGetUniqueId");
        static_assert(sizeof(u) == VR_COMM_ID_BYTES, "RCCL unique id size");
        std::memcpy(id, &u, sizeof u);
        return VR_OK;
    });
}

int vr_create_multi_ex(const float* voxels, int32_t voxels_on_device, int64_t d1, int64_t d2, int64_t d3,
                       double cal_max, const vr_tf_interval* tf, int32_t n_tf, const int32_t* devices, int32_t n_gpus,
                       const vr_options* options, vr_ctx** out) {
    if (!out) return VR_EINVAL;
    *out = nullptr;
    if (!voxels || !devices || n_gpus <= 0 || n_gpus > 64) return VR_EINVAL;
    return guard([&] {
        const size_t count = checked_count(d1, d2, d3);
        std::vector<int> dev(devices, devices + n_gpus);
        // transports: RCCL between distinct GPUs; a list that repeats a GPU moves the tiles with
        // hipMemcpyPeerAsync (RCCL refuses two ranks on one device).  Only a list of ONE GPU repeated
        // is a valid rehearsal: a mixed list ({0, 1, 1}) would need both (its peer-copy events and
        // streams would sit on different GPUs), and is refused before anything is created.
        std::vector<int> sorted(dev);
        std::sort(sorted.begin(), sorted.end());
        const bool repeats = std::adjacent_find(sorted.begin(), sorted.end()) != sorted.end();
        if (repeats && sorted.front() != sorted.back())
            throw Error(VR_EINVAL, "vr_create_multi: a device list either names distinct GPUs or repeats one GPU");
        int ndev = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) throw Error(VR_ENODEV, "vr_create_multi: no GPU");
        for (int d : dev)
            if (d < 0 || d >= ndev) throw Error(VR_ENODEV, "vr_create_multi: bad device index");
        std::unique_ptr<vr_ctx, int (*)(vr_ctx*)> c(create_common(voxels, voxels_on_device != 0, d1, d2, d3, cal_max,
                                                                  tf, n_tf, dev[0], options), vr_destroy);
        Group* g = new_group(c.get(), n_gpus, 0);
        c->group = g;
        g->peer_copy = repeats;
        if (n_gpus > 1 && !g->peer_copy) {
            g->comms.assign((size_t)n_gpus, nullptr);
            nccl_check(ncclCommInitAll(g->comms.data(), n_gpus, dev.data()), "ncclCommInitAll");
        }
        std::vector<DevBuf> bufs((size_t)n_gpus);
        for (int i = 1; i < n_gpus; ++i) {
            hip_check(hipSetDevice(dev[(size_t)i]));
            bufs[(size_t)i].ensure(count * sizeof(float));
        }
        if (n_gpus > 1) broadcast_volume(g, c.get(), dev, bufs, count);
        for (int i = 1; i < n_gpus; ++i) {
            hip_check(hipSetDevice(dev[(size_t)i]));
            g->parts.push_back(create_common(nullptr, true, d1, d2, d3, cal_max, tf, n_tf, dev[(size_t)i], options,
                                             &bufs[(size_t)i]));
            g->parts.back()->part_of = g;
        }
        *out = c.release();
        return VR_OK;
    });
}

int vr_create_multi(const float* voxels, int64_t d1, int64_t d2, int64_t d3, double cal_max, const vr_tf_interval* tf,
                    int32_t n_tf, const int32_t* devices, int32_t n_gpus, const vr_options* options, vr_ctx** out) {
    return vr_create_multi_ex(voxels, 0, d1, d2, d3, cal_max, tf, n_tf, devices, n_gpus, options, out);
}

int vr_create_rank(const float* voxels, int32_t voxels_on_device, int64_t d1, int64_t d2, int64_t d3, double cal_max,
                   const vr_tf_interval* tf, int32_t n_tf, int32_t device, int32_t rank, int32_t n_ranks,
                   const uint8_t comm_id[VR_COMM_ID_BYTES], const vr_options* options, vr_ctx** out) {
    if (!out) return VR_EINVAL;
    *out = nullptr;
    if (!comm_id || n_ranks <= 0 || n_ranks > 64 || rank < 0 || rank >= n_ranks || (rank == 0 && !voxels))
        return VR_EINVAL;
    return guard([&] {
        // a rank that threw between ncclCommInitRank and the broadcast would leave its peers blocked
        // inside the broadcast: argument and device checks come first, and an allocation failure is
        // carried into the agreement below instead of thrown
        const size_t count = checked_count(d1, d2, d3);
        int ndev = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) throw Error(VR_ENODEV, "vr_create_rank: no GPU");
        if (device < 0 || device >= ndev) throw Error(VR_ENODEV, "vr_create_rank: bad device index");
        hip_check(hipSetDevice(device));
        // the agreement buffer and the stream first (tiny), then the volume, whose allocation may fail
        // on one rank only: that rank still joins the communicator and the agreement, so every rank
        // learns of the failure and none is left inside a collective
        DevBuf agree;
        agree.ensure(10 * sizeof(double));
        hipStream_t st = nullptr;
        hip_check(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        DevBuf vol;
        double ok = 1.0;
        try {
            vol.ensure(count * sizeof(float));
        } catch (...) {
            ok = 0.0;
        }
        ncclUniqueId u;
        std::memcpy(&u, comm_id, sizeof u);
        ncclComm_t comm = nullptr;
        try {
            nccl_check(ncclCommInitRank(&comm, n_ranks, u, rank), "ncclCommInitRank");
        } catch (...) {
            (void)hipStreamDestroy(st);
            throw;
        }
        vr_ctx* c = nullptr;
        try {
            // agreement, one ncclAllReduce(MAX) of (v, -v) for v = (d1, d2, d3, cal_max, ok) before any
            // broadcast: every rank must hold its buffers, and every rank's dims and cal_max must be
            // rank 0's (the max and the min of a value agree only if all ranks passed the same)
            const double h[10] = {(double)d1, (double)d2, (double)d3, cal_max, ok,
                                  -(double)d1, -(double)d2, -(double)d3, -cal_max, -ok};
            double r[10];
            hip_check(hipMemcpyAsync(agree.p, h, sizeof h, hipMemcpyHostToDevice, st));
            nccl_check(ncclAllReduce(agree.p, agree.p, 10, ncclFloat64, ncclMax, comm, st), "ncclAllReduce (agreement)");
            hip_check(hipMemcpyAsync(r, agree.p, sizeof r, hipMemcpyDeviceToHost, st));
            rank_wait(st, comm, options, "the creation agreement (ncclAllReduce)");
            if (-r[9] != 1.0) throw Error(VR_ENOMEM, "vr_create_rank: a rank could not allocate the volume");
            for (int i = 0; i < 4; ++i)
                if (r[i] != -r[5 + i]) throw Error(VR_EINVAL, "vr_create_rank: ranks disagree on the volume dims / cal_max");
            if (rank == 0)
                hip_check(hipMemcpyAsync(vol.p, voxels, count * sizeof(float),
                                         voxels_on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, st));
            const size_t chunk = (size_t)1 << 28;   // 1 GiB pieces
            for (size_t o = 0; o < count; o += chunk) {
                const size_t n = std::min(chunk, count - o);
                nccl_check(ncclBroadcast(vol.as<float>() + o, vol.as<float>() + o, n, ncclFloat32, 0, comm, st),
                           "ncclBroadcast (volume)");
            }
            rank_wait(st, comm, options, "the volume broadcast");
            hip_check(hipStreamDestroy(st));
            st = nullptr;
            c = create_common(nullptr, true, d1, d2, d3, cal_max, tf, n_tf, device, options, &vol);
        } catch (...) {
            if (st) {
                (void)hipStreamSynchronize(st);   // (an aborted communicator's kernels have exited)
                (void)hipStreamDestroy(st);
            }
            if (comm) (void)ncclCommDestroy(comm);
            throw;
        }
        Group* g = new_group(c, n_ranks, rank);
        g->comms.push_back(comm);
        c->group = g;
        *out = c;
        return VR_OK;
    });
}

int vr_group_info(vr_ctx* c, int32_t* n_gpus, int32_t* rank, int32_t* transport) {
    if (!c) return VR_EINVAL;
    const Group* g = c->group;
    if (n_gpus) *n_gpus = g ? g->n_ranks : 1;
    if (rank) *rank = g ? g->rank0 : 0;
    if (transport) *transport = !g || g->n_ranks == 1 ? VR_TRANSPORT_NONE : g->peer_copy ? VR_TRANSPORT_PEER_COPY
                                                                                       : VR_TRANSPORT_RCCL;
    return VR_OK;
}

int vr_group_timing_read(vr_ctx* c, int32_t rank, double* total_ms, int64_t* launches, int32_t reset) {
    if (!c) return VR_EINVAL;
    return guard([&] {
        const Group* g = c->group;
        vr_ctx* pc = c;
        if (g) {
            // one-process groups hold every part; a vr_create_rank context only its own rank
            const int i = rank - g->rank0;
            if (i < 0 || i >= (int)g->parts.size()) throw Error(VR_EINVAL, "vr_group_timing_read: rank not held here");
            pc = g->parts[(size_t)i];
        } else if (rank != 0) {
            throw Error(VR_EINVAL, "vr_group_timing_read: a one-GPU context has rank 0 only");
        }
        set_device(pc);
        drain_timing(pc);
        if (total_ms) *total_ms = pc->timing_ms;
        if (launches) *launches = pc->timing_launches;
        if (reset) { pc->timing_ms = 0; pc->timing_launches = 0; }
        return VR_OK;
    });
}

int vr_group_traffic_read(vr_ctx* c, int32_t rank, int64_t* bytes_sent, int64_t* bytes_received, int64_t* frames,
                          int32_t reset) {
    if (!c) return VR_EINVAL;
    Group* g = c->group;
    int64_t tx = 0, rx = 0, fr = 0;
    if (g) {
        const int i = rank - g->rank0;   // (as vr_group_timing_read: a part held by this context)
        if (i < 0 || i >= (int)g->parts.size()) return VR_EINVAL;
        if ((size_t)i < g->tx_bytes.size()) {
            tx = g->tx_bytes[(size_t)i];
            rx = g->rx_bytes[(size_t)i];
            fr = g->tx_frames[(size_t)i];
            if (reset) g->tx_bytes[(size_t)i] = g->rx_bytes[(size_t)i] = g->tx_frames[(size_t)i] = 0;
        }
    } else if (rank != 0) {
        return VR_EINVAL;
    }
    if (bytes_sent) *bytes_sent = tx;
    if (bytes_received) *bytes_received = rx;
    if (frames) *frames = fr;
    return VR_OK;
}

int vr_group_tiles(vr_ctx* c, int32_t rank, int32_t* tiles, int32_t capacity, int32_t* n_out) {
    if (!c || !n_out || capacity < 0) return VR_EINVAL;
    const Group* g = c->group;
    if (!g) { *n_out = 0; return VR_OK; }
    if (rank < 0 || rank >= g->n_ranks) return VR_EINVAL;
    if (!g->last) { *n_out = 0; return VR_OK; }
    const std::vector<int32_t>& L = g->last->lists[(size_t)rank];
    *n_out = (int32_t)L.size();
    if (tiles) std::copy(L.begin(), L.begin() + std::min<size_t>(L.size(), (size_t)capacity), tiles);
    return VR_OK;
}

}  // extern "C"
