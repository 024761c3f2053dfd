/*
 * vr_api.h -- C-ABI of the MI355X-native direct-volume ray marcher (libvr.so).
 *
 * This is the drop-in boundary for the reference's `namespace myCUDAspace` (kernel.h:15-75), the
 * C++ API renderLoop (myApp.cu:789-1074) calls.  Plain pointers and sizes only; no C++ or torch
 * types.  Every entry point below names the reference call(s) it replaces.
 *
 * Conventions (reference: kernel.h:31-74, myApp.cu:1066-1072)
 *   - Status: every function returns 0 on success or a negative VR_E* code; vr_strerror() gives
 *     a message (a HIP failure keeps the hipError_t text).  Where the reference returned
 *     cudaError_t and printed to stderr, we return the code and print nothing.
 *   - Ownership: the caller owns every host buffer.  vr_create* copies the volume to the GPU; the
 *     context owns all device memory until vr_destroy (reference: allocateDeviceMemory2 /
 *     deallocateDeviceMemory with T** out-params).
 *   - Threading: a context is used from one host thread.  A one-GPU context (vr_create*) is bound
 *     to its `device`; a multi-GPU context drives several GPUs behind the same calls -- one process
 *     for all of them (vr_create_multi) or one process per GPU (vr_create_rank) -- and farms the
 *     screen tiles and gathers them into rank 0 over RCCL itself (see the multi-GPU section below
 *     and INTEGRATION.md).  vr_render_tiles / vr_assemble_* remain for callers that farm tiles
 *     with their own transport.
 *   - Synchronous by default like the reference (it called cudaDeviceSynchronize in every
 *     wrapper); vr_render_tiles with VR_OUT_ASYNC returns after enqueueing on the ctx stream.
 *   - Frame layout: out[(x*H + y)*4 + c], float32 RGBA, x-major (blendSampleColors, kernel.cu:203,
 *     :222); alpha is forced to 1 like the reference.
 */
#ifndef VR_API_H
#define VR_API_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VR_API_VERSION 3

/* ---- status codes ------------------------------------------------------------------------- */
#define VR_OK 0
#define VR_EINVAL (-1)     /* bad argument (null pointer, size, mode, flags)                   */
#define VR_EIO (-2)        /* file missing / unreadable / not NIfTI (reference continued!)      */
#define VR_EFORMAT (-3)    /* NIfTI datatype or dimensionality not supported                   */
#define VR_ENOMEM (-4)     /* host or device allocation failed                                 */
#define VR_EHIP (-5)       /* a HIP runtime call failed; vr_strerror has the hipError_t text   */
#define VR_ENODEV (-6)     /* no GPU / bad device index                                        */
#define VR_ERANGE (-7)     /* volume or frame too large for the requested mode                 */
#define VR_ECOMM (-8)      /* multi-GPU contexts: an RCCL call failed, or a wait on a part passed
                              vr_options.comm_timeout_ms; the communicators are aborted and every
                              later render call fails the same way (vr_destroy still works; until
                              then queued work may still write the call's output)              */

/* ---- render modes (utils.h:13-18 algorithm IDs) ------------------------------------------- */
#define VR_MODE_VRC 1      /* octree-leaf nearest sampling (kernel.cu:40-70)                   */
#define VR_MODE_TEST 5     /* classify-then-trilinear over the raw grid (kernel.cu:72-187)     */

/* ---- render flags -------------------------------------------------------------------------- */
#define VR_FLAG_ESS 1      /* empty-space skipping (bitwise exact: skips only alpha-0 samples)  */
#define VR_FLAG_ERT 2      /* front-to-back + early ray termination at T < ert_epsilon          */
#define VR_FLAG_SHADE 8    /* opt-in central-difference gradient + headlight Phong (no reference) */
#define VR_FLAG_CONIC 16   /* perspective rays: dir = normalize(screen point - camera pos), sample
                              = pos + (s*sd + fc)*dir (kernel.cu:30-34, :53-54; the reference ships
                              it disabled, utils.h:28).  Use vr_camera_derive_conic's top_left.  */
/* Without VR_FLAG_ERT the march is back to front exactly like blendSampleColors. */

/* ---- output flags (vr_render's out_flags, vr_render_tiles / vr_assemble_tiles) ------------- */
#define VR_OUT_DEVICE 1    /* vr_render: out_rgba is device memory of the context's GPU         */
#define VR_OUT_ASYNC 2     /* enqueue only on the ctx stream; caller synchronises (vr_synchronize) */
#define VR_OUT_RGB 4       /* tile buffers (vr_render_tiles / _tile_list, vr_assemble_tiles / _tile_list):
                              3 floats per pixel, r g b -- alpha is 1 by construction (kernel.cu:213),
                              so the gathered bytes drop by a quarter; assembly writes alpha = 1   */

typedef struct vr_ctx vr_ctx;

/* Camera after processInput's re-derivation (myApp.cu:1106-1112) -- AppData camera fields,
 * utils.h:41-46 and :68-70.  Passed by value per frame (replaces updateCameraLocation +
 * updateDeviceAppdataCameraKernel, kernel.cu:1111-1123, :251-260). */
typedef struct {
    float pos[3], front[3], right[3], up[3], top_left[3];
} vr_camera;

/* One TransferFunction interval (TransferFunction.h:15-19): closed [lo, hi] -> material colour.
 * Order matters: the LAST interval containing the value wins, default interval 0
 * (TransferFunction.cu:46-55). */
typedef struct {
    float lo, hi;
    float rgba[4];
} vr_tf_interval;

/* AppData render fields (utils.h:36-74) made runtime.  vr_params_default fills the reference's
 * values for a given W, H, S. */
typedef struct {
    int32_t width, height, samples_per_ray, mode, flags;
    float real_screen_width, real_screen_height, viewplane_distance, front_clip_plane,
        sample_distance;
    float background[4];
    float ert_epsilon;     /* VR_FLAG_ERT only; 1e-5 keeps frames within 1e-4 of exact        */
    float shade_ambient, shade_diffuse, shade_specular, shade_shininess; /* VR_FLAG_SHADE only */
} vr_params;

/* Volume statistics of a context (read-only). */
typedef struct {
    int64_t dim[3];
    double cal_max;
    uint32_t longest_dimension, octree_depth;   /* Octree.cu:35-41 */
    int32_t n_tf;
    int32_t zero_transparent;                   /* TF(0).a == 0: clipping + ESS are exact      */
    uint64_t device_bytes;                      /* device memory held by the context           */
    int32_t idx64;                              /* 1: 64-bit class-volume offsets (>= 2^31 B)  */
    int32_t reserved;
    uint64_t class_bytes;                       /* VRC class volume (u8, bricked and padded)    */
} vr_volume_info;

/* Tuning options of a context.  The defaults (vr_options_default) are the measured best on
 * MI355X; the other values exist for A/B measurement and for parity tests
 * of paths the defaults only take at other sizes.  None of them changes a frame's values: every
 * setting renders the same frame (ESS / ERT tolerances aside, which vr_params selects).
 * Layout fields are fixed when the context is created (vr_create_ex); the render fields may be
 * changed between frames with vr_set_options.  The library reads no environment variables. */
typedef struct {
    /* layout (vr_create_ex only) */
    int32_t brick[3];          /* class-volume brick, voxels per axis (default 4 x 4 x 8)            */
    int32_t cell_shift;        /* macro cell = 2^cell_shift octree leaves per axis; -1 = auto        */
    int32_t force_idx64;       /* 64-bit class offsets even below 2^31 class bytes (parity tests)   */
    /* render */
    int32_t batch;             /* samples per straight-line batch per lane: 0 = auto, 8 or 16        */
    int32_t cull;              /* whole-frame screen-space culling of off-volume work tiles: 0 off,
                                  1 outside the projected dataset box's bounding rectangle, 2 (default)
                                  also the work tiles of that rectangle off the box's projected hull
                                  (general views).  Culled pixels are exactly the background.      */
    int32_t view_table_reuse;  /* axis-aligned views: reuse the per-view sample table (1)            */
    int32_t work_order;        /* work-tile -> XCD deal: 0 diagonal (default; TEST frames of general
                                  views interleave whole tile columns), 1 sectors, 2 columns        */
    int32_t axis_table;        /* axis-aligned views use the per-frame sample table march (1)        */
    int32_t occ_lds;           /* stage the occupancy bitmask in LDS when it fits (1)                */
    int32_t persist_wgs;       /* persistent grid, workgroups per CU; 0 = one workgroup per tile     */
    /* multi-GPU contexts (render) */
    int32_t farm_tile;         /* screen tile edge in pixels, a multiple of 16 (default 64)           */
    float farm_rank0_weight;   /* rank 0's share of the tiles relative to each other rank (default 1)*/
    /* render */
    int32_t leaf_map_pad;      /* general orthographic views: padded LDS leaf maps, no per-sample
                                  clamps (1); 0 = clamped lookups.  Bitwise the same frames.         */
    int32_t exact_skip;        /* exact (back-to-front, no ERT) orthographic frames skip empty macro
                                  cells (1): bitwise the same frames, alpha-0 samples being exact
                                  no-ops of the back-to-front blend; 0 = march every sample          */
    int32_t frames_in_flight;  /* vr_render_batch: consecutive frames rotate over 1 + frames_in_flight
                                  HIP streams (0..3; default 1: two), so one frame's march tail
                                  overlaps the next ones' starts                                     */
    int32_t test_plane_march;  /* TEST frames along a volume axis carry their corner planes from
                                  sample to sample (1; test_axis_kernel): bitwise the same frames     */
    int32_t comm_timeout_ms;   /* multi-GPU contexts: longest wait on a part's stream or an RCCL
                                  operation before every communicator is aborted and the call fails
                                  with VR_ECOMM (default 60000; 0 = wait forever)                    */
    int32_t class_bits;        /* bits per voxel class in the VRC class volume: 0 = auto (the fewest of
                                  2 / 4 / 8 that hold the TF's classes; default), or 2, 4, 8 (raised
                                  to what the TF needs).  Smaller classes = a smaller, cache-resident
                                  volume; bitwise the same frames                                    */
    int32_t run_words;         /* axis-aligned views along z: a batch's classes from the two aligned
                                  8-byte words of its first and last samples (2 loads per batch, not
                                  one per sample); 0 = auto (64-bit-offset volumes), 1 = off, 2 = on.
                                  Bitwise the same frames                                          */
    int32_t table_split;       /* axis-aligned views along z: per-sample view-table entries hold the
                                  class byte and bit apart (1, default: one add and one bit-field
                                  extract per gather); 0 = bit offsets.  Bitwise the same frames    */
    /* layout (vr_create_ex only) */
    int32_t test_corners;      /* TEST frames of general views read a sample's 8 trilinear corner classes
                                  in ONE gather from a corner volume: 0 (default) = per voxel the 8
                                  classes at the TF's class width (16 bits for <= 4 intervals, 32 for
                                  <= 16, else 64) in the reference's x-major order; 3 = the same in
                                  4 x 4 x 4-voxel bricks; 1 = 64 bits per voxel, x-major; 2 = none
                                  (four corner-row gathers per sample).  Exact frames bitwise the
                                  same in every mode; front to back (VR_FLAG_ERT) with <= 4 intervals,
                                  modes 0 and 3 read a 16-KB plane table instead of the TF and agree
                                  with modes 1 and 2 within the ERT tolerance                       */
    int32_t leaf_columns;      /* axis-aligned ESS marches read the empty-cell mask of the ray's own leaf
                                  column (1, default, up to 2048 leaves per axis) instead of its 4 x 4-
                                  leaf cell column (0).  Device memory per classification (every TF
                                  change): a transient one-bit-per-leaf occupancy, nleaf^3 / 8 bytes
                                  (2048 leaves: 1 GiB), and 3 nleaf^2 64-bit masks kept (2048: 100 MB;
                                  the MNI shape, 256 leaves: 1.5 MB).  Bitwise the same frames       */
} vr_options;

int vr_options_default(vr_options* out);

/* ---- lifecycle ---------------------------------------------------------------------------- */

/* Copies an x-major float32 volume (index x*d2*d3 + y*d3 + z, BinaryLoader.cu:234-238) and the
 * transfer function to GPU `device`; builds the leaf maps, classification and occupancy
 * pyramid there.  Replaces allocateDeviceMemory2 (kernel.cu:876-1068) + Octree construction
 * (Octree.cu:30-53, host 0.3-2.8 s in the reference). */
int vr_create(const float* voxels, int64_t d1, int64_t d2, int64_t d3, double cal_max,
              const vr_tf_interval* tf, int32_t n_tf, int32_t device, vr_ctx** out);

/* Same, but the voxels are already in device memory of `device` (e.g. received over RCCL);
 * the context copies them (device-to-device). */
int vr_create_from_device(const float* d_voxels, int64_t d1, int64_t d2, int64_t d3,
                          double cal_max, const vr_tf_interval* tf, int32_t n_tf,
                          int32_t device, vr_ctx** out);

/* vr_create / vr_create_from_device (voxels_on_device != 0) with explicit options (NULL = the
 * defaults). */
int vr_create_ex(const float* voxels, int32_t voxels_on_device, int64_t d1, int64_t d2, int64_t d3,
                 double cal_max, const vr_tf_interval* tf, int32_t n_tf, int32_t device,
                 const vr_options* options, vr_ctx** out);
/* Reads / changes a context's options.  vr_set_options changes the render fields only; the
 * layout fields must equal the context's (VR_EINVAL otherwise). */
int vr_get_options(vr_ctx* ctx, vr_options* out);
int vr_set_options(vr_ctx* ctx, const vr_options* options);

/* ---- multi-GPU contexts (the reference runs on device 0 only, kernel.cu:885) ---- *
 * A multi-GPU context renders with vr_render like any other: the visible 64 x 64 screen tiles
 * (vr_visible_tiles) are dealt to its GPUs interleaved (rank 0 weighted by
 * vr_options.farm_rank0_weight), each GPU marches its tiles, the tiles are gathered into rank 0's
 * GPU over xGMI (RCCL ncclSend / ncclRecv, one link per peer) and one assembly launch writes the
 * frame there.  Frames are bitwise those of a one-GPU context.  The volume is copied to rank 0's
 * GPU and RCCL-broadcast to the others once; every GPU builds its own classes and tables.
 * vr_set_transfer_function, vr_set_options and vr_synchronize apply to every GPU of a
 * single-process group; the other entry points that take a context (tiles, assembly, egress,
 * counts, timing, info) act on rank 0's GPU. */
#define VR_COMM_ID_BYTES 128
#define VR_TRANSPORT_NONE 0        /* one GPU                                                      */
#define VR_TRANSPORT_RCCL 1        /* ncclSend / ncclRecv over xGMI                                */
#define VR_TRANSPORT_PEER_COPY 2   /* hipMemcpyPeerAsync (a device list that repeats a GPU: RCCL
                                      refuses two ranks on one device; rehearsals of the plan)     */

/* One process drives n_gpus GPUs (devices[0] is rank 0; one RCCL communicator per GPU,
 * ncclCommInitAll).  The list names distinct GPUs, or repeats ONE GPU n_gpus times (a rehearsal of
 * the n-part plan moving tiles with hipMemcpyPeerAsync); a mixed list such as {0, 1, 1} is VR_EINVAL.  The other GPUs of a C++ host: replaces the single-device
 * allocateDeviceMemory2 (kernel.cu:876-1068). */
int vr_create_multi(const float* voxels, int64_t d1, int64_t d2, int64_t d3, double cal_max,
                    const vr_tf_interval* tf, int32_t n_tf, const int32_t* devices, int32_t n_gpus,
                    const vr_options* options, vr_ctx** out);
/* One process per GPU (torchrun / MPI style).  Rank 0 calls vr_comm_unique_id and hands the id
 * to every rank (any channel: MPI_Bcast, a file, torch.distributed); every rank then calls
 * vr_create_rank (collectively: it blocks until all ranks have joined) with the same dims,
 * cal_max and TF; only rank 0 passes voxels (host memory, or device memory of its GPU with
 * voxels_on_device = 1), which are RCCL-broadcast.  Every rank
 * must call vr_render for every frame with the same params and camera; rank 0's out receives the
 * frame, the others may pass NULL. */
int vr_comm_unique_id(uint8_t id[VR_COMM_ID_BYTES]);
int vr_create_rank(const float* voxels, int32_t voxels_on_device, int64_t d1, int64_t d2, int64_t d3,
                   double cal_max, const vr_tf_interval* tf, int32_t n_tf, int32_t device, int32_t rank,
                   int32_t n_ranks, const uint8_t comm_id[VR_COMM_ID_BYTES], const vr_options* options,
                   vr_ctx** out);
/* vr_create_multi with the voxels in device memory of devices[0] (voxels_on_device = 1), e.g. a
 * volume generated on the GPU (the 34.4 GB C5 replica never exists on the host). */
int vr_create_multi_ex(const float* voxels, int32_t voxels_on_device, int64_t d1, int64_t d2, int64_t d3,
                       double cal_max, const vr_tf_interval* tf, int32_t n_tf, const int32_t* devices,
                       int32_t n_gpus, const vr_options* options, vr_ctx** out);
/* The group a context belongs to: GPUs, this context's rank, VR_TRANSPORT_*. */
int vr_group_info(vr_ctx* ctx, int32_t* n_gpus, int32_t* rank, int32_t* transport);
/* vr_timing_read for one GPU of a group: part `rank` of a one-process group (vr_timing_enable
 * enables every part), or a vr_create_rank context's own rank. */
int vr_group_timing_read(vr_ctx* ctx, int32_t rank, double* total_ms, int64_t* launches, int32_t reset);
/* The peer traffic of part `rank` (held by this context, as vr_group_timing_read) since its last
 * reset: the tile bytes it posted to rank 0 over the transport, the bytes it posted to receive
 * (rank 0: every peer's tiles), and the frames it took part in.  `reset` clears that part's
 * counters only.  A one-GPU context reports zeros for rank 0.  (bench.py prints the per-frame figures beside DESIGN section 7's
 * predicted ones.) */
int vr_group_traffic_read(vr_ctx* ctx, int32_t rank, int64_t* bytes_sent, int64_t* bytes_received,
                          int64_t* frames, int32_t reset);
/* The tile ids rank `rank` rendered in the last frame (x-major, farm_tile-sized tiles). */
int vr_group_tiles(vr_ctx* ctx, int32_t rank, int32_t* tiles, int32_t capacity, int32_t* n_out);

/* Loads a NIfTI-2/-1 file (BinaryLoader.cu:273-335, but fails hard on a missing or malformed
 * file instead of continuing with an uninitialised header) and calls vr_create. */
int vr_create_from_nifti(const char* path, const vr_tf_interval* tf, int32_t n_tf,
                         int32_t device, vr_ctx** out);

/* Replaces the transfer function (TransferFunction ctor, TransferFunction.cu:8-39);
 * re-classifies on the GPU. */
int vr_set_transfer_function(vr_ctx* ctx, const vr_tf_interval* tf, int32_t n_tf);

/* deallocateDeviceMemory (kernel.cu:1072-1093). */
int vr_destroy(vr_ctx* ctx);

/* ---- rendering ---------------------------------------------------------------------------- */

/* Renders one W x H frame.  Replaces the per-frame sequence updateCameraLocation ->
 * updatePrimaryRayDirection -> getSampleColors | getSampleColorsFromNF -> blendSampleColors ->
 * cudaMemcpy D2H (myApp.cu:883-915, :988-1011) with ONE fused kernel (no W*H*S sample
 * buffer).  out_rgba: W*H*4 floats in host memory (out_flags = 0, synchronous like the
 * reference) or device memory of the context's GPU (VR_OUT_DEVICE, optionally | VR_OUT_ASYNC). */
int vr_render(vr_ctx* ctx, const vr_params* params, const vr_camera* camera, float* out_rgba,
              int32_t out_flags);

/* n_frames frames with the same params, frame f seen by cameras[f] (a moving camera), written to
 * out_frames + f*W*H*4 (out_flags as vr_render).  Equal to n_frames vr_render calls; on a
 * multi-GPU context the batch's tiles reach rank 0 in ONE RCCL group and ONE scatter launch, so
 * the host cost of the collective is paid once per batch.  On a one-process-per-GPU group every
 * rank calls it with the same cameras; ranks other than 0 may pass NULL. */
int vr_render_batch(vr_ctx* ctx, const vr_params* params, const vr_camera* cameras, int32_t n_frames,
                    float* out_frames, int32_t out_flags);

/* Renders the screen tiles t = first_tile + k*tile_stride (k = 0, 1, ...) of a W x H frame cut
 * into tile_w x tile_h tiles numbered x-major (t = tx*ntiles_y + ty).  Output is a compact
 * device buffer d_tiles[k][tile_w*tile_h][4] (VR_OUT_RGB: [3]) with pixel (i, j) of a tile at i*tile_h + j;
 * pixels outside the frame are left untouched.  For multi-GPU screen-tile farming: rank r of N
 * passes first_tile = r, tile_stride = N.  *n_tiles_out = number of tiles written. */
int vr_render_tiles(vr_ctx* ctx, const vr_params* params, const vr_camera* camera,
                    int32_t tile_w, int32_t tile_h, int32_t first_tile, int32_t tile_stride,
                    float* d_tiles, int32_t* n_tiles_out, int32_t out_flags);

/* Scatters gathered compact tile buffers into an x-major frame on the device:
 * d_tiles holds, for rank r = 0..n_ranks-1, a block of max_tiles_per_rank tiles (the layout of
 * vr_render_tiles with first_tile = r, tile_stride = n_ranks).  d_frame: W*H*4 floats. */
int vr_assemble_tiles(vr_ctx* ctx, int32_t width, int32_t height, int32_t tile_w, int32_t tile_h,
                      int32_t n_ranks, int32_t max_tiles_per_rank, const float* d_tiles,
                      float* d_frame, int32_t out_flags);

/* Screen-space culling for tile farming: the ids (x-major, t = tx*nty + ty) of the tiles of a
 * tile_w x tile_h grid that can hold a non-background pixel -- a conservative bound of the
 * projected dataset box, widened by 2 pixels (VRC, orthographic or conic, TF(0) transparent;
 * otherwise every tile).  Every other pixel is exactly params->background.  Writes up to
 * `capacity` ids (ascending) into tiles (may be NULL) and the total into *n_tiles_out. */
int vr_visible_tiles(vr_ctx* ctx, const vr_params* params, const vr_camera* camera, int32_t tile_w,
                     int32_t tile_h, int32_t* tiles, int32_t capacity, int32_t* n_tiles_out);

/* vr_render_tiles over an explicit list of tile ids (host array of n_tiles): renders
 * tiles[first], tiles[first + stride], ... into the compact buffer d_tiles (same layout). */
int vr_render_tile_list(vr_ctx* ctx, const vr_params* params, const vr_camera* camera, int32_t tile_w,
                        int32_t tile_h, const int32_t* tiles, int32_t n_tiles, int32_t first,
                        int32_t stride, float* d_tiles, int32_t* n_tiles_out, int32_t out_flags);

/* Assembly for a tile list: block k of rank r in d_tiles (max_tiles_per_rank blocks per rank)
 * holds tile tiles[r + k*n_ranks]; every pixel of a tile not in the list is set to background. */
int vr_assemble_tile_list(vr_ctx* ctx, int32_t width, int32_t height, int32_t tile_w, int32_t tile_h,
                          const int32_t* tiles, int32_t n_tiles, int32_t n_ranks,
                          int32_t max_tiles_per_rank, const float* d_tiles, const float background[4],
                          float* d_frame, int32_t out_flags);

/* Assembly for an explicit tile -> block assignment (weighted multi-GPU plans, where ranks hold
 * different numbers of tiles): tile tiles[i] is block slots[i] of d_tiles (n_blocks blocks of
 * tile_w*tile_h pixels, 4 or -- VR_OUT_RGB -- 3 floats each); every pixel of a tile not listed is
 * set to background.  Replaces the host-side frame stitching the reference never needed (one GPU). */
int vr_assemble_tile_slots(vr_ctx* ctx, int32_t width, int32_t height, int32_t tile_w, int32_t tile_h,
                           const int32_t* tiles, const int32_t* slots, int32_t n_tiles, int32_t n_blocks,
                           const float* d_tiles, const float background[4], float* d_frame,
                           int32_t out_flags);

/* vr_assemble_tile_slots for a batch of n_frames frames in one launch: frame f takes tile tiles[i]
 * from block slots[f*n_tiles + i] and is written to d_frames + f*W*H*4 (frames back to back). */
int vr_assemble_tile_slots_multi(vr_ctx* ctx, int32_t width, int32_t height, int32_t tile_w, int32_t tile_h,
                                 const int32_t* tiles, const int32_t* slots, int32_t n_tiles, int32_t n_frames,
                                 int32_t n_blocks, const float* d_tiles, const float background[4],
                                 float* d_frames, int32_t out_flags);

/* Number of samples of the frame whose octree leaf lies inside the dataset (the N_in of the
 * algorithmic-bytes model), counted exactly on the GPU. */
int vr_count_samples(vr_ctx* ctx, const vr_params* params, const vr_camera* camera,
                     uint64_t* n_in_dataset);

/* Work the march actually does for one frame (the bench's roofline numerator): renders the frame
 * once on the context's GPU (the first part of a multi-GPU context) with vr_render's work list,
 * options and kernel variant -- empty-space skipping and early termination as the params select --
 * and returns the class gathers that touched memory (*gathers: 1 byte each) and the samples
 * evaluated (*samples, optional: batches x batch length, skipped samples excluded).  VRC only.
 * A diagnostic pass (two atomics per ray): never inside a timed region. */
int vr_count_marched(vr_ctx* ctx, const vr_params* params, const vr_camera* camera, uint64_t* gathers,
                     uint64_t* samples);

/* vr_count_marched for either mode, with the bytes: the march's class gathers that touched memory,
 * the bytes they read at their own widths (VRC: 1 B per class byte, 16 B per batch of run words;
 * TEST: 2 / 4 / 8 B per corner-volume entry, 4 B per corner-row dword, 32 B per z-window of the axis
 * march) and the samples evaluated.  The same kernel variant as vr_render, in its counting
 * instantiation (atomics per ray): never inside a timed region. */
typedef struct {
    uint64_t gathers;
    uint64_t bytes;
    uint64_t samples;
    uint64_t reserved;
} vr_work_count;
int vr_count_work(vr_ctx* ctx, const vr_params* params, const vr_camera* camera, vr_work_count* out);

int vr_synchronize(vr_ctx* ctx);
/* Use an external HIP stream (hipStream_t passed as void*); NULL restores the ctx's own.  Work on the
   new stream starts after everything queued on the old one.  A single-GPU ctx releases its own
   stream when given an external one (HIP shares a few hardware queues among a process's streams; an
   idle stream still takes a share) and recreates it on NULL. */
int vr_set_stream(vr_ctx* ctx, void* hip_stream);

/* ---- frame egress ------------------------------------------------------ */
#define VR_ORIENT_RAW 0            /* img[y][x]                                                    */
#define VR_ORIENT_VRC_DISPLAY 1    /* img[y][W-1-x]: the VRC window as saved by saveImage          */
#define VR_ORIENT_TEST_DISPLAY 2   /* img[H-1-y][x]: the TEST window as saved by saveImage         */
/* Replaces transformSScreenVec4toFloat (myApp.cu:1661-1688) + the GL draw (VRC rotated 180 deg
 * about z, myApp.cu:933) + glReadPixels/stbi_flip_vertically_on_write (myApp.cu:1942-1956) for a
 * headless box: the device frame d_frame (x-major float RGBA, as vr_render writes it) becomes H
 * rows of W RGB8 pixels, top row first, each channel round(clamp(c, 0, 1) * 255).  rgb is a
 * device buffer if out_flags has VR_OUT_DEVICE, else host memory (the call then synchronises). */
int vr_frame_to_rgb8(vr_ctx* ctx, int32_t width, int32_t height, int32_t orientation,
                     const float* d_frame, uint8_t* rgb, int32_t out_flags);
/* vr_render into the context's own device frame, then vr_frame_to_rgb8 and vr_write_png: the
 * headless saveImage of a rendered frame (myApp.cu:1203-1221, :1942-1956) for a C / C++ host that
 * holds no device memory of its own.  VR_EIO when the file cannot be written. */
int vr_render_png(vr_ctx* ctx, const vr_params* params, const vr_camera* camera, int32_t orientation,
                  const char* path);
/* PNG file (8-bit RGB, deflate) of H rows of W RGB8 pixels, top row first (saveImage's output
 * format).  VR_EIO when the file cannot be written. */
int vr_write_png(const char* path, int32_t width, int32_t height, const uint8_t* rgb);

/* ---- POINT mode ------------------------------------------------------- */
/* prepareVolumeColors (myApp.cu:1280-1316) on the GPU: writes d1*d2*d3*7 floats into the device
 * buffer d_out, voxel (x,y,z) at ((x*d2 + y)*d3 + z)*7: position ((v + L/2) - d/2) / L per axis
 * (L = longest dimension), then the RGBA of TF(voxel / cal_max).  The vertex layout the reference
 * uploads to its POINT VBO. */
int vr_point_cloud(vr_ctx* ctx, float* d_out, int32_t out_flags);

/* ---- workloads ------------------------------------------------------------------------------ */
/* The synthetic n^3 float32 volume of SURVEY 8(d) C5 (n = 2048, seed 0x5EED there), generated on
 * GPU `device` into d_out for the x-slab [x0, x0 + nx): d_out[((x-x0)*n + y)*n + z].
 * c = (n-1)/2, r = |(x,y,z) - c| / (n/2); for r < 0.95
 * v = clamp(round(127.5 + 127.5 sin(16 pi r)) + splitmix64(seed ^ ((x*n + y)*n + z)) % 17 - 8, 0, 255),
 * else 0.  Double precision.  Runs on hip_stream (NULL: the null stream) and synchronises. */
int vr_synthetic_volume(float* d_out, int64_t n, int64_t x0, int64_t nx, uint64_t seed, int32_t device,
                        void* hip_stream);

/* ---- host helpers (AppData / processInput restated, glm-identical float arithmetic) -------- */

/* utils.h:53-74 for a W x H x S frame: rsw = 2 tan(pi/4), rsh = rsw*H/W, vpd = 2, fc = 0,
 * sd = (vpd - fc)/S, background (.2,.2,.2,1); mode VRC, flags 0. */
int vr_params_default(int32_t width, int32_t height, int32_t samples_per_ray, vr_params* out);
/* processInput's re-derivation with no key pressed (myApp.cu:1105-1112) from pos and the
 * current up vector. */
int vr_camera_derive(const float pos[3], const float up[3], float real_screen_width,
                     float real_screen_height, vr_camera* out);
/* The conic variant of the camera update (utils.h:93-97, commented-out initialiser utils.h:62-66):
 * as vr_camera_derive, but top_left = pos + vpd*front + (rsw/2)*(-right) + up*(rsh/2).  For conic
 * frames the reference sizes the screen as rsw = 2 tan(view_angle) * vpd (utils.h:57). */
int vr_camera_derive_conic(const float pos[3], const float up[3], float real_screen_width,
                           float real_screen_height, float viewplane_distance, vr_camera* out);
/* The steady default camera: AppData initialisers (utils.h:41-46) + one processInput pass. */
int vr_camera_default(int32_t width, int32_t height, vr_camera* out);
/* The reset camera of key X (utils.h:77-81, resetCameraAttributes myApp.cu:1911-1917). */
int vr_camera_reset(vr_camera* out);
/* The reference's transfer function (TransferFunction.cu:19-23, Material.cpp:6-67); returns
 * the number of intervals written (4); out must hold >= 4. */
int vr_default_transfer_function(vr_tf_interval* out, int32_t capacity);

/* NiftiFile loader on its own (no GPU): fills dims[3] and *cal_max; if voxels != NULL also copies
 * dims[0]*dims[1]*dims[2] float32 values (x-major) into it.  Same hardening as
 * vr_create_from_nifti. */
int vr_nifti_read(const char* path, int64_t dims[3], double* cal_max, float* voxels);
/* OctreeHandler's closed-form leaf grid (Octree.cu:79-129) for a d1 x d2 x d3 volume: writes
 * 3 * 2^D int32 (per axis, leaf -> voxel index or -1) into maps if capacity allows, and the depth
 * D into *depth.  Returns the number of entries (3 * 2^D). */
int vr_octree_leaf_maps(int64_t d1, int64_t d2, int64_t d3, int32_t* maps, int64_t capacity,
                        uint32_t* depth);

/* ---- introspection / measurement ---------------------------------------------------------- */
int vr_get_volume_info(vr_ctx* ctx, vr_volume_info* out);
/* HIP-event timing of the march kernel(s) on the ctx stream: enable, then read the summed
 * kernel milliseconds and launch count since the last reset (vr_timing_read synchronises the
 * stream; events are recorded around every march launch without host synchronisation). */
int vr_timing_enable(vr_ctx* ctx, int32_t enable);
int vr_timing_read(vr_ctx* ctx, double* total_ms, int64_t* launches, int32_t reset);
const char* vr_strerror(int status);
int vr_device_count(int32_t* count);
int vr_api_version(void);

#ifdef __cplusplus
}
#endif
#endif /* VR_API_H */
