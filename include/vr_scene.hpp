// vr_scene.hpp -- public C++ host API of libvr.so, keeping the reference's host-side nouns so a
// C++ application written against them (myApp.cu main, renderLoop) finds the same classes:
//   NiftiFile          BinaryLoader.h:16-51, BinaryLoader.cu:273-415
//   Material           Material.h:14-37, Material.cpp:6-67
//   TransferFunction   TransferFunction.h:15-39, TransferFunction.cu:8-55
//   OctreeHandler      OctreeHandler.h:6-10 (an empty class in the reference); here the builder of
//                      the implicit octree's leaf grid (Octree.cu:30-129) in closed form
//   VolumeRenderer     RAII owner of a vr_ctx (include/vr_api.h): allocateDeviceMemory2 + the
//                      per-frame myCUDAspace calls + deallocateDeviceMemory (kernel.h:31-74)
// The classes are compiled into libvr.so (default visibility); VolumeRenderer is header-only over
// the C-ABI.  Link with -lvr.  Differences from the reference: NiftiFile throws vr::Error (status
// code + message) on a missing or malformed file instead of continuing with an uninitialised
// header (BinaryLoader.cu:333); TransferFunction::size() is a method over a std::vector.
#pragma once
#include <cstdint>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "vr_api.h"

namespace vr {

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

// ---------------------------------------------------------------------------------------------
// NIfTI-2 / NIfTI-1 volume.  The reference (BinaryLoader.cu:273-335) reads the 540-byte header
// raw and dim1*dim2*dim3 float32 from vox_offset, ignoring datatype and scl_*; a missing file only
// prints "Unable to open file" and continues with an uninitialised header.  This loader fails
// hard, accepts NIfTI-1 (348-byte) and byte-swapped headers, and converts integer / float64
// datatypes to float32.  Values are kept raw (scl_slope is ignored, as in the reference) so a
// float32 file renders identically.
// ---------------------------------------------------------------------------------------------
class NiftiFile {
public:
    struct Header {
        int32_t sizeof_hdr = 540;
        int16_t datatype = 16, bitpix = 32;
        int64_t dim[8] = {3, 0, 0, 0, 1, 1, 1, 1};
        double pixdim[8] = {0, 1, 1, 1, 1, 1, 1, 1};
        int64_t vox_offset = 544;
        double scl_slope = 0, scl_inter = 0, cal_max = 0, cal_min = 0;
    };

    explicit NiftiFile(const std::string& filename);
    NiftiFile(std::vector<float> volume, int64_t d1, int64_t d2, int64_t d3, double cal_max);

    Header header;
    std::vector<float> volume;
    int longest_dimension = 0;   // BinaryLoader.cu:33-36 (max over dims)
    int64_t totaldim = 0;        // setTotalDim, BinaryLoader.cu:409-415

    // BinaryLoader.cu:234-238: (int)x * d2 * d3 + (int)y * d3 + (int)z  (int64 here)
    int64_t transformVector3Position(float x, float y, float z) const {
        return (int64_t)(int)x * header.dim[2] * header.dim[3] + (int64_t)(int)y * header.dim[3] + (int)z;
    }
    // BinaryLoader.cu:240-245
    bool isInside(float x, float y, float z) const {
        return x >= 0.0f && x < (float)header.dim[1] && y >= 0.0f && y < (float)header.dim[2] &&
               z >= 0.0f && z < (float)header.dim[3];
    }

private:
    void finish();
};

// ---------------------------------------------------------------------------------------------
// Material / TransferFunction (Material.h:14-37, TransferFunction.h:15-40)
// ---------------------------------------------------------------------------------------------
namespace Material {
struct Material {
    const char* name;
    float color[4];                       // rgba
    double Henyey_Greenstein_scattering;  // carried, unused on the render path (as in the reference)
};
enum MaterialId { red, green, blue, bone, muscle, eye, brain, cerebelum, cerebrospinal_fluid, brain_stem,
                  glass, empty, air, default_ };
Material getMaterialFromID(MaterialId id);   // Material.cpp:6-67
}  // namespace Material

struct MatInterval {   // mat_interval, TransferFunction.h:15-19
    Material::Material material;
    float lower_bound, higher_bound;
};

class TransferFunction {
public:
    TransferFunction();                                  // the reference TF, TransferFunction.cu:8-39
    explicit TransferFunction(std::vector<MatInterval> intervals);
    // TransferFunction.cu:46-55: default interval 0; the LAST closed interval containing value wins.
    int getMaterialIndex(float value) const;
    const Material::Material* getMaterial(float value) const {
        return &material_intervals[getMaterialIndex(value)].material;
    }
    std::vector<MatInterval> material_intervals;
    int size() const { return (int)material_intervals.size(); }
};

// ---------------------------------------------------------------------------------------------
// OctreeHandler: closed form of the implicit octree's leaf grid (Octree.cu:30-129).
// Leaf i (lower corner i / 2^D on every axis, dyadic-exact in float) is scaled by L and accepted
// on axis a iff L/2 - d_a/2 <= L*lc < L/2 + d_a/2; its voxel is (int)(L*lc + d_a/2 - L/2).  The
// acceptance and voxel index are separable per axis, so the leaf grid is the tensor product of
// three maps leaf -> voxel (or -1 = outside the dataset -> value 0).
// ---------------------------------------------------------------------------------------------
struct OctreeHandler {
    uint32_t longest_dimension = 0;   // L, Octree.cu:35-38
    uint32_t maximum_depth = 0;       // D = ceil(log2 L), Octree.cu:40-41
    uint64_t number_of_nodes = 0;     // the reference's node count (sum 8^p), for reporting
    int32_t nleaf = 0;                // 2^D
    std::vector<int32_t> maps;        // 3 * nleaf: [axis][leaf] -> voxel or -1
    int32_t leaf_lo[3] = {0, 0, 0}, leaf_hi[3] = {-1, -1, -1};   // accepted leaf range per axis

    void build(int64_t d1, int64_t d2, int64_t d3);
};

// ---------------------------------------------------------------------------------------------
// VolumeRenderer: one vr_ctx, i.e. the volume + transfer function resident on the GPU(s).
// ---------------------------------------------------------------------------------------------
class VolumeRenderer {
public:
    // allocateDeviceMemory2 (kernel.cu:876-1068): the volume and TF to GPU `device`
    VolumeRenderer(const NiftiFile& nf, const TransferFunction& tf, int device = 0) {
        const std::vector<vr_tf_interval> iv = intervals(tf);
        check(vr_create(nf.volume.data(), nf.header.dim[1], nf.header.dim[2], nf.header.dim[3], nf.header.cal_max,
                        iv.data(), (int32_t)iv.size(), device, &ctx_), "vr_create");
    }
    // the same over several GPUs of this process (screen tiles farmed, gathered over RCCL)
    VolumeRenderer(const NiftiFile& nf, const TransferFunction& tf, const std::vector<int32_t>& devices) {
        const std::vector<vr_tf_interval> iv = intervals(tf);
        check(vr_create_multi(nf.volume.data(), nf.header.dim[1], nf.header.dim[2], nf.header.dim[3],
                              nf.header.cal_max, iv.data(), (int32_t)iv.size(), devices.data(),
                              (int32_t)devices.size(), nullptr, &ctx_), "vr_create_multi");
    }
    VolumeRenderer(const VolumeRenderer&) = delete;
    VolumeRenderer& operator=(const VolumeRenderer&) = delete;
    VolumeRenderer(VolumeRenderer&& o) noexcept : ctx_(o.ctx_) { o.ctx_ = nullptr; }
    ~VolumeRenderer() { vr_destroy(ctx_); }   // deallocateDeviceMemory (kernel.cu:1072-1093)

    // getSampleColors / getSampleColorsFromNF + blendSampleColors + the D2H copy
    // (myApp.cu:883-915): host frame [(x*H + y)*4 + c], alpha 1
    std::vector<float> render(const vr_params& p, const vr_camera& cam) {
        std::vector<float> frame((size_t)p.width * p.height * 4);
        check(vr_render(ctx_, &p, &cam, frame.data(), 0), "vr_render");
        return frame;
    }
    // the frame as the reference's window shows it, saved like saveImage (myApp.cu:1942-1956)
    void render_png(const vr_params& p, const vr_camera& cam, const std::string& path,
                    int32_t orientation = VR_ORIENT_VRC_DISPLAY) {
        check(vr_render_png(ctx_, &p, &cam, orientation, path.c_str()), "vr_render_png");
    }
    void set_transfer_function(const TransferFunction& tf) {
        const std::vector<vr_tf_interval> iv = intervals(tf);
        check(vr_set_transfer_function(ctx_, iv.data(), (int32_t)iv.size()), "vr_set_transfer_function");
    }
    vr_ctx* handle() const { return ctx_; }

    static std::vector<vr_tf_interval> intervals(const TransferFunction& tf) {
        std::vector<vr_tf_interval> iv;
        for (const MatInterval& m : tf.material_intervals)
            iv.push_back({m.lower_bound, m.higher_bound,
                          {m.material.color[0], m.material.color[1], m.material.color[2], m.material.color[3]}});
        return iv;
    }

private:
    static void check(int rc, const char* what) {
        if (rc < 0) throw Error(rc, std::string(what) + ": " + vr_strerror(rc));
    }
    vr_ctx* ctx_ = nullptr;
};

}  // namespace vr
