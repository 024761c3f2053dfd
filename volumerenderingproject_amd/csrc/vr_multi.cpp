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
#include <cstring>

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
    int n_ranks = 1;                      // ranks of the group (GPUs)
    int rank0 = 0;                        // global rank of parts[0] (multi-process: this process's rank)
    std::vector<vr_ctx*> parts;           // parts[0] = the owning context (not owned here), others owned
    std::vector<ncclComm_t> comms;        // one per part; empty for the peer-copy transport / one rank
    bool peer_copy = false;               // single process over repeated devices: hipMemcpyPeerAsync
    int tile = 64;
    float w0 = 1.0f;                      // rank 0's weight in the tile deal (others 1)
    std::vector<DevBuf> send;             // per part: its tiles, compact RGB (rank 0 renders into recv)
    DevBuf recv;                          // rank 0: the gathered tiles, rank-major blocks
    std::vector<hipEvent_t> copied;       // peer copy: part i's buffer consumed by rank 0's stream
    std::vector<hipEvent_t> ready;        // peer copy: part i's tiles rendered
    std::vector<bool> copied_pending;
    // plan of the last frame (recomputed when the visible tile list changes)
    int W = -1, H = -1;
    std::vector<int32_t> ids;             // visible tiles, ascending
    std::vector<std::vector<int32_t>> lists;   // per global rank
    std::vector<int64_t> off;             // per global rank: first block in recv
    std::vector<int32_t> tiles, slots;    // assembly map: tile tiles[i] is block slots[i]
};

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

void plan(Group* g, int W, int H, std::vector<int32_t>&& ids) {
    if (W == g->W && H == g->H && ids == g->ids) return;
    g->W = W; g->H = H;
    g->ids = std::move(ids);
    g->lists = weighted_lists(g->ids, g->n_ranks, g->w0);
    g->off.assign((size_t)g->n_ranks + 1, 0);
    g->tiles.clear(); g->slots.clear();
    for (int r = 0; r < g->n_ranks; ++r) {
        g->off[(size_t)r + 1] = g->off[(size_t)r] + (int64_t)g->lists[(size_t)r].size();
        for (size_t k = 0; k < g->lists[(size_t)r].size(); ++k) {
            g->tiles.push_back(g->lists[(size_t)r][k]);
            g->slots.push_back((int32_t)(g->off[(size_t)r] + (int64_t)k));
        }
    }
}

void sync_all(Group* g) {
    for (vr_ctx* pc : g->parts) {
        set_device(pc);
        hip_check(hipStreamSynchronize(pc->stream));
    }
}

Group* new_group(vr_ctx* c, int n_ranks, int rank0) {
    Group* g = new Group;
    g->n_ranks = n_ranks;
    g->rank0 = rank0;
    g->w0 = c->opt.farm_rank0_weight;
    g->tile = c->opt.farm_tile;
    g->parts.push_back(c);
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
    hip_check(hipStreamSynchronize(root->stream));   // the root's volume copy has landed
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
    }
    for (size_t i = 0; i < devices.size(); ++i) {
        hip_check(hipSetDevice(devices[i]));
        hip_check(hipStreamSynchronize(st[i]));
        hip_check(hipStreamDestroy(st[i]));
    }
}

}  // namespace

void group_destroy(Group* g) {
    if (!g) return;
    for (vr_ctx* pc : g->parts) {
        (void)hipSetDevice(pc->device);
        (void)hipStreamSynchronize(pc->stream);
    }
    for (size_t i = 0; i < g->copied.size(); ++i) {
        (void)hipSetDevice(g->parts[i]->device);
        if (g->copied[i]) (void)hipEventDestroy(g->copied[i]);
        if (g->ready[i]) (void)hipEventDestroy(g->ready[i]);
    }
    for (ncclComm_t cm : g->comms)
        if (cm) (void)ncclCommDestroy(cm);
    g->recv.reset();
    for (size_t i = 0; i < g->send.size(); ++i) {
        (void)hipSetDevice(g->parts[i]->device);
        g->send[i].reset();
    }
    for (size_t i = 1; i < g->parts.size(); ++i) destroy_ctx_single(g->parts[i]);
    delete g;
}

void group_options_changed(vr_ctx* c) {
    Group* g = c->group;
    if (!g) return;
    sync_all(g);
    g->w0 = c->opt.farm_rank0_weight;
    g->tile = c->opt.farm_tile;
    g->W = g->H = -1;   // re-plan at the next frame
}

void group_for_each(vr_ctx* c, void (*fn)(vr_ctx*, void*), void* arg) {
    if (!c->group) {
        fn(c, arg);
        return;
    }
    for (vr_ctx* pc : c->group->parts) fn(pc, arg);
}

void group_render(vr_ctx* c, const vr_params* p, const vr_camera* cam, float* out, int32_t out_flags) {
    Group* g = c->group;
    const int T = g->tile;
    const bool holds_rank0 = g->rank0 == 0;
    const bool out_on_device = (out_flags & VR_OUT_DEVICE) != 0;
    if (holds_rank0 && !out) throw Error(VR_EINVAL, "vr_render: rank 0 of a multi-GPU context needs an output");
    // the plan: every rank derives the same visible-tile list from the same camera (no exchange)
    plan(g, p->width, p->height, visible_tiles(c, p, cam, T, T));
    const size_t per = (size_t)T * T * 3;   // floats per RGB tile (alpha is 1 by construction)
    const int n_parts = (int)g->parts.size();
    if (g->send.size() != (size_t)n_parts) {
        g->send = std::vector<DevBuf>((size_t)n_parts);
        g->copied.assign((size_t)n_parts, nullptr);
        g->ready.assign((size_t)n_parts, nullptr);
        g->copied_pending.assign((size_t)n_parts, false);
    }
    if (holds_rank0) {
        set_device(c);
        g->recv.ensure(std::max<size_t>(1, (size_t)g->off[(size_t)g->n_ranks]) * per * sizeof(float));
    }
    // 1. every part marches its tiles (asynchronously, on its own stream and GPU)
    for (int i = 0; i < n_parts; ++i) {
        vr_ctx* pc = g->parts[(size_t)i];
        const int gr = g->rank0 + i;
        const std::vector<int32_t>& mine = g->lists[(size_t)gr];
        if (mine.empty()) continue;
        set_device(pc);
        float* dst;
        if (gr == 0) {
            dst = g->recv.as<float>();
        } else {
            g->send[(size_t)i].ensure(mine.size() * per * sizeof(float));
            if (g->copied_pending[(size_t)i]) {   // peer copy: the previous frame's copy has read the buffer
                hip_check(hipStreamWaitEvent(pc->stream, g->copied[(size_t)i], 0));
                g->copied_pending[(size_t)i] = false;
            }
            dst = g->send[(size_t)i].as<float>();
        }
        render_tile_list(pc, p, cam, T, T, mine, dst, 1);
    }
    // 2. the peers' tiles into rank 0
    if (g->n_ranks > 1) {
        if (g->peer_copy) {
            set_device(c);
            for (int i = 1; i < n_parts; ++i) {
                vr_ctx* pc = g->parts[(size_t)i];
                const size_t n = g->lists[(size_t)i].size();
                if (!n) continue;
                set_device(pc);
                if (!g->ready[(size_t)i]) hip_check(hipEventCreateWithFlags(&g->ready[(size_t)i], hipEventDisableTiming));
                if (!g->copied[(size_t)i]) hip_check(hipEventCreateWithFlags(&g->copied[(size_t)i], hipEventDisableTiming));
                hip_check(hipEventRecord(g->ready[(size_t)i], pc->stream));
                set_device(c);
                hip_check(hipStreamWaitEvent(c->stream, g->ready[(size_t)i], 0));
                hip_check(hipMemcpyPeerAsync(g->recv.as<float>() + (size_t)g->off[(size_t)i] * per, c->device,
                                             g->send[(size_t)i].as<float>(), pc->device, n * per * sizeof(float),
                                             c->stream));
                hip_check(hipEventRecord(g->copied[(size_t)i], c->stream));
                g->copied_pending[(size_t)i] = true;
            }
        } else {
            nccl_check(ncclGroupStart(), "ncclGroupStart");
            for (int i = 0; i < n_parts; ++i) {
                vr_ctx* pc = g->parts[(size_t)i];
                const int gr = g->rank0 + i;
                if (gr != 0) {
                    const size_t n = g->lists[(size_t)gr].size();
                    if (n)
                        nccl_check(ncclSend(g->send[(size_t)i].as<float>(), n * per, ncclFloat32, 0,
                                            g->comms[(size_t)i], pc->stream), "ncclSend (tiles)");
                } else {
                    for (int q = 1; q < g->n_ranks; ++q) {
                        const size_t n = g->lists[(size_t)q].size();
                        if (n)
                            nccl_check(ncclRecv(g->recv.as<float>() + (size_t)g->off[(size_t)q] * per, n * per,
                                                ncclFloat32, q, g->comms[(size_t)i], pc->stream), "ncclRecv (tiles)");
                    }
                }
            }
            nccl_check(ncclGroupEnd(), "ncclGroupEnd");
        }
    }
    // 3. rank 0 assembles the frame (gathered tiles where listed, the background elsewhere)
    if (holds_rank0) {
        set_device(c);
        const size_t bytes = (size_t)p->width * p->height * sizeof(float4);
        float* dst = out;
        if (!out_on_device) {
            c->frame.ensure(bytes);
            dst = c->frame.as<float>();
        }
        assemble_slots(c, p->width, p->height, T, T, g->tiles, g->slots,
                       (int)std::max<int64_t>(1, g->off[(size_t)g->n_ranks]), g->recv.as<float>(), p->background,
                       dst, 1);
        if (!out_on_device) hip_check(hipMemcpyAsync(out, dst, bytes, hipMemcpyDeviceToHost, c->stream));
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

int vr_create_multi(const float* voxels, int64_t d1, int64_t d2, int64_t d3, double cal_max, const vr_tf_interval* tf,
                    int32_t n_tf, const int32_t* devices, int32_t n_gpus, const vr_options* options, vr_ctx** out) {
    if (!out) return VR_EINVAL;
    *out = nullptr;
    if (!voxels || !devices || n_gpus <= 0 || n_gpus > 64) return VR_EINVAL;
    return guard([&] {
        int ndev = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) throw Error(VR_ENODEV, "vr_create_multi: no GPU");
        std::vector<int> dev(devices, devices + n_gpus);
        for (int d : dev)
            if (d < 0 || d >= ndev) throw Error(VR_ENODEV, "vr_create_multi: bad device index");
        std::unique_ptr<vr_ctx, int (*)(vr_ctx*)> c(create_common(voxels, false, d1, d2, d3, cal_max, tf, n_tf, dev[0],
                                                                  options), vr_destroy);
        Group* g = new_group(c.get(), n_gpus, 0);
        c->group = g;
        std::vector<int> sorted(dev);
        std::sort(sorted.begin(), sorted.end());
        g->peer_copy = std::adjacent_find(sorted.begin(), sorted.end()) != sorted.end();
        if (n_gpus > 1 && !g->peer_copy) {
            g->comms.assign((size_t)n_gpus, nullptr);
            nccl_check(ncclCommInitAll(g->comms.data(), n_gpus, dev.data()), "ncclCommInitAll");
        }
        const size_t count = (size_t)(d1 * d2 * d3);
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
        }
        *out = c.release();
        return VR_OK;
    });
}

int vr_create_rank(const float* voxels, int64_t d1, int64_t d2, int64_t d3, double cal_max, const vr_tf_interval* tf,
                   int32_t n_tf, int32_t device, int32_t rank, int32_t n_ranks, const uint8_t comm_id[VR_COMM_ID_BYTES],
                   const vr_options* options, vr_ctx** out) {
    if (!out) return VR_EINVAL;
    *out = nullptr;
    if (!comm_id || n_ranks <= 0 || rank < 0 || rank >= n_ranks || (rank == 0 && !voxels)) return VR_EINVAL;
    return guard([&] {
        int ndev = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) throw Error(VR_ENODEV, "vr_create_rank: no GPU");
        if (device < 0 || device >= ndev) throw Error(VR_ENODEV, "vr_create_rank: bad device index");
        hip_check(hipSetDevice(device));
        ncclUniqueId u;
        std::memcpy(&u, comm_id, sizeof u);
        ncclComm_t comm = nullptr;
        nccl_check(ncclCommInitRank(&comm, n_ranks, u, rank), "ncclCommInitRank");
        const size_t count = (size_t)(d1 * d2 * d3);
        vr_ctx* c = nullptr;
        try {
            DevBuf vol;
            hipStream_t st;
            hip_check(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
            if (rank == 0) {
                vol.ensure(count * sizeof(float));
                hip_check(hipMemcpyAsync(vol.p, voxels, count * sizeof(float), hipMemcpyHostToDevice, st));
            } else {
                vol.ensure(count * sizeof(float));
            }
            const size_t chunk = (size_t)1 << 28;   // 1 GiB pieces
            for (size_t o = 0; o < count; o += chunk) {
                const size_t n = std::min(chunk, count - o);
                nccl_check(ncclBroadcast(vol.as<float>() + o, vol.as<float>() + o, n, ncclFloat32, 0, comm, st),
                           "ncclBroadcast (volume)");
            }
            hip_check(hipStreamSynchronize(st));
            hip_check(hipStreamDestroy(st));
            c = create_common(nullptr, true, d1, d2, d3, cal_max, tf, n_tf, device, options, &vol);
        } catch (...) {
            (void)ncclCommDestroy(comm);
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

int vr_group_tiles(vr_ctx* c, int32_t rank, int32_t* tiles, int32_t capacity, int32_t* n_out) {
    if (!c || !n_out || capacity < 0) return VR_EINVAL;
    const Group* g = c->group;
    if (!g) { *n_out = 0; return VR_OK; }
    if (rank < 0 || rank >= g->n_ranks) return VR_EINVAL;
    if (g->lists.empty()) { *n_out = 0; return VR_OK; }
    const std::vector<int32_t>& L = g->lists[(size_t)rank];
    *n_out = (int32_t)L.size();
    if (tiles) std::copy(L.begin(), L.begin() + std::min<size_t>(L.size(), (size_t)capacity), tiles);
    return VR_OK;
}

}  // extern "C"
