// vr_device.h -- shared host/device structures of the HIP ray marcher (internal, not the ABI).
#pragma once
#include <stdint.h>

namespace vr {

// Workgroup = 256 lanes = 16 x 16 rays; each wave64 covers an 8 x 8 ray block.
constexpr int kWgRaysX = 16;
constexpr int kWgRaysY = 16;
constexpr int kWgThreads = 256;
// march geometry variants; kGeomAxis1Run = kGeomAxis1 with the run-word class gathers (VrcFrame.zrun),
// kGeomAxis1Z = kGeomAxis1 along z with the split {byte, bit} view table (VrcFrame.tsplit)
constexpr int kGeomOrtho = 0, kGeomAxis1 = 1, kGeomConic = 2, kGeomAxis1Run = 3, kGeomAxis1Z = 4;
constexpr int kMaxTf = 256;
constexpr int kLeafColsMax = 2048;   // leaf-column masks (AXIS1 ESS) up to this many leaves per axis
constexpr int kBgGroup = 8;         // culled whole-frame work tiles stored per background-only workgroup
constexpr int kCellDistCap = 16;   // cap of the ESS Chebyshev cell-distance field (relaxation steps)
constexpr int kMaxTabSamples = 8192;   // AXIS1 per-frame sample table (LDS) up to this many samples per ray
constexpr int kMaxTestTab = 4096;      // TEST general views: per-frame B table (16 B per entry, <= 64 KB LDS)
constexpr int kMaxHull = 8;         // edges of the projected dataset box's hull (workgroup cull)
// general views: a leaf outside the dataset is -2^29 in the staged leaf maps, so for class volumes
// under 2^29 units the sum of the three contributions is negative -- an out-of-range buffer offset --
// whenever one of them is outside
constexpr int32_t kMapOut = -(1 << 29);
// general 32-bit views: the leaf maps in global memory carry kMapPadMax kMapOut entries either side
// of each axis (pmaps_pad), so a frame's LDS maps with pad <= kMapPadMax are one contiguous copy
constexpr int kMapPadMax = 64;
// zero bytes after the TEST class volume: the corner-row dword gathers may read up to 3 bytes past
// the last voxel (class 0 there IS the reference's idx < total guard); the buffer bound is total +
// kClsPad / 4, so even an in-range dword at the bound stays inside the allocation
constexpr int kClsPad = 64;

// One workgroup's work tile: rays [x0, x0+16) x [y0, y0+16).  In tile-output mode `slot` is the
// compact user-tile slot and (tox, toy) the work tile's offset inside that user tile.
struct WorkTile {
    int32_t x0, y0, slot, tofs;   // tofs = (tox << 16) | toy
};

// worklist_kernel's occupancy cull of an axis-parallel orthographic whole frame (vr_api.cpp
// frame_list): a work tile all of whose rays' cell columns along the view axis are empty is exactly
// the background.  sat = the column table of that axis (occupied columns in [0, u) x [0, v), side x
// side), nullptr = no cull; the two fixed axes' top-left / right / up components in double.
struct WlCull {
    const int32_t* sat;
    int32_t side, cb_shift, nleaf, W, H;
    double tl[2], right[2], up[2];
    double rsw, rsh;
};

// Per-frame constants of the VRC march, passed by value (kernarg segment -> SGPRs).
struct VrcFrame {
    // screen / camera (AppData fields, utils.h:36-74; camera after processInput)
    int32_t W, H, S, flags;
    float rsw, rsh, sd, fc;
    float tlc[3], right[3], up[3], front[3];
    float bg[4];
    float ert_eps;
    // volume (leaf grid of the implicit octree, Octree.cu:35-49)
    int64_t d2d3, d3;
    int32_t depth;          // D
    float leaves;           // 2^D
    int32_t cb_shift;       // macro cell = 2^cb_shift leaves per axis
    int32_t ncell;          // macro cells per axis
    float cell_q;           // macro cell edge in q units (2^cb_shift / 2^D)
    float shrink_q;         // ESS safety shrink, q units
    float step[3];          // q advance per sample = sd * front (per frame: rays are parallel)
    float inv_step[3];      // 1 / step (0 where step == 0)
    int32_t occ_words;      // 32-bit words of the occupancy bitmask
    int32_t occ_lds;        // bitmask staged in LDS
    int32_t axis1;          // index of the only non-zero component of front (axis-aligned view), else -1
    float box_lo[3], box_hi[3];   // dataset box in q space (+margin), for clipping
    int edge_guard;               // marched samples may leave the unit cube (ESS must not jump there)
    int conic;                    // VR_FLAG_CONIC: rays from campos through the screen point
    float campos[3];
    int32_t zero_transparent;     // TF(0).a == 0
    int32_t cls0;                 // class of TF(0 / (float)(int)cal_max): outside cube / dataset
    int32_t nleaf;                // 2^D (leaf-map length per axis)
    // output
    int32_t out_tiles;            // 0: frame [x*H+y]; 1: compact tiles
    int32_t out_rgb;              // compact tiles of 3 floats per pixel (VR_OUT_RGB)
    int32_t tile_w, tile_h;
    int32_t n_work;               // entries in the work list
    int32_t n_slots;              // entries in the block order (>= grid size)
    int32_t persist_wgs;          // > 0: persistent launch with this many workgroups per CU
    int32_t cls_bytes;            // class volume bytes when < 2^31 (buffer-resource bound of the gathers)
    // class addressing (32-bit volumes): offsets are bits when cbits < 8 -- the class is the cbits-wide
    // field at bit (o & omask) of byte o >> osh -- and bytes at 8 bits (osh = omask = 0)
    int32_t cbits, osh, omask;
    int32_t mapout_ok;            // offsets stay below 2^29 units: a kMapOut term makes any sum negative
    // AXIS1 run words (views along z): a batch's classes come from the two aligned 8-byte words that
    // hold its first and last samples; qsh = log2(units per word) (6 bits, 3 bytes), bsh = log2(bits
    // per unit) (0, 3).  0: one class load per sample
    int32_t zrun, qsh, bsh;
    int32_t zspan2;               // zrun: every batch spans at most two z-bricks (host bound on the step)
    int32_t tsplit;               // AXIS1 along z, 32-bit volume: view-table entries {byte offset, bit}
    int32_t c0_noop;              // TF class 0 has alpha 0: its premultiplied entry (0, 0, 0, 1) is a no-op
    int32_t bg_first;             // whole frames: first culled entry of the work list (n_work: none)
    int32_t bg_group;             // culled entries per background-only workgroup (blocks >= bg_first)
    int32_t pad;                  // general views: kMapOut entries either side of each LDS leaf map (0: none)
    int32_t leafcols;             // AXIS1 + ESS: occcol holds leaf-column masks (3 nleaf^2), else cell-column masks
    // whole frames, general views: the projected dataset box's hull, edge e keeping the pixels with
    // hull[e][0] x + hull[e][1] y <= hull[e][2] (vr_api.cpp hull_edges); 0 edges = no claim
    int32_t n_hull;
    float hull[kMaxHull][3];
    // shading (VR_FLAG_SHADE)
    float ka, kd, ks, shininess;
    int32_t d1i, d2i, d3i;        // dims as int for gradient clamping
};

// Per-frame constants of the TEST march (kernel.cu:72-187).
struct TestFrame {
    int32_t W, H, S, flags;
    float mc[16], iv[16], tv[16];   // modelCam, inverse(lookAt), toVolume; column-major
    float bg[4];
    float ert_eps;
    int64_t d1, d2, d3, total;
    float fd1, fd2, fd3;
    int32_t zero_transparent;
    int32_t cls0;                   // class of TF(0 / cal_max)
    int32_t out_tiles, tile_w, tile_h, n_work;
    int32_t out_rgb;                // compact tiles of 3 floats per pixel (VR_OUT_RGB)
    int32_t idx64;                  // 64-bit corner indices (total + d2*d3 + d3 >= 2^31)
    int32_t tcb, tnc[3];            // ESS macro cells: 2^tcb voxels per axis, cells per axis
    int32_t occ_words, occ_lds;
    int32_t sep;                    // mc and tv are axis-separable (scale + translate): see test_march_kernel
    int32_t sep_tab;                // sep + the per-frame B table fits its LDS budget (S + 8 <= kMaxTestTab)
    int32_t axt;                    // -1, or the volume axis a along which the rays march with the other two
                                    // coordinates of p fixed (test_axis_kernel; make_test's conditions)
    int32_t axt_up;                 // p_a grows with s (tv_aa * iv_{8+a} * mc10 > 0)
    int32_t ax_sb, ax_se;           // axis views: the clip range [ax_sb, ax_se) of every ray whose (p_b, p_c)
                                    // lies in the volume -- p_a(s) is the same for every ray (make_test)
    // axis views: per corner line (the two other coordinates, each in [0, d + 2)) a 64-bit mask over
    // cells of tca[a] voxels along a (tnca[a] <= 64 cells): bit c = a byte of the line's flat
    // indices at a in [c tca, c tca + tca + 1] (the corners a sample whose (int)p_a lies in cell c
    // reads) has alpha > 0 (test_columns_kernel); line (u, v) at tcol_base[a] + u tcol_pitch[a] + v
    int32_t tca[3], tnca[3], tcol_pitch[3];
    int64_t tcol_base[3];
    int32_t cv;                     // the general march's corner volume (test_corner_kernel): 0 none; CB = 2 / 4 / 8
                                    // bits per corner class in 4^3-voxel bricks, 16 + CB x-major
    int32_t cv_bytes;               // its bytes (< 2^31: the gathers' buffer bound)
    int32_t mul24;                  // d1 and d2 d3 < 2^24: x-major corner offsets in 24-bit multiplies
    float wthr[3];                  // 1 - ulp(d_a + 1): a fraction below it has (int)(p + 1) == (int)p + 1
    int32_t lin;                    // every voxel on the volume's six faces is class 0: the general march's
                                    // trilinear colour is continuous across the faces (test_faces_kernel)
    int32_t bg_first;               // whole frames: first background-only workgroup (INT32_MAX: none)
    int32_t bg_group;               // culled work tiles per background-only workgroup
    int32_t n_hull;                 // general views: the projected dataset box's hull (VrcFrame.hull)
    float hull[kMaxHull][3];
};

// TransferFunction::getMaterial (TransferFunction.cu:46-55): last closed interval containing v, else 0
__device__ __forceinline__ int tf_class(const float* lo, const float* hi, int n, float v) {
    int r = 0;
    for (int i = 0; i < n; ++i)
        if (v >= lo[i] && v <= hi[i]) r = i;
    return r;
}

}  // namespace vr
