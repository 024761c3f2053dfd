// scene.h -- C++ host model of the render path, keeping the reference's API nouns:
//   NiftiFile          (BinaryLoader.h:16-51, BinaryLoader.cu)
//   Material / TransferFunction (Material.h, Material.cpp, TransferFunction.h, TransferFunction.cu)
//   OctreeHandler      (the north star's name for the octree builder; OctreeHandler.h:6-10 is an
//                       empty class in the reference) -- here it derives the implicit octree's leaf
//                       grid (Octree.cu:30-129) in closed form: per-axis leaf -> voxel maps.
//   Camera helpers     (AppData utils.h:24-82, processInput myApp.cu:1105-1112, TEST matrices
//                       kernel.cu:1177-1216)
#pragma once
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "glm_float.h"

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
// Camera / AppData helpers
// ---------------------------------------------------------------------------------------------
struct CameraState {
    glmf::vec3 pos, front, right, up, top_left;
};
// utils.h:58-59, :74
void default_screen(int W, int H, int S, float* rsw, float* rsh, float* vpd, float* fc, float* sd);
// myApp.cu:1105-1112 with identity rotation/translation
CameraState derive_camera(glmf::vec3 pos, glmf::vec3 up, float rsw, float rsh);
CameraState derive_camera_conic(glmf::vec3 pos, glmf::vec3 up, float rsw, float rsh, float vpd);
CameraState default_camera(int W, int H);
CameraState reset_camera();
// kernel.cu:1177-1216
void test_matrices(int64_t d1, int64_t d2, int64_t d3, int W, int H, int S, float rsw, float rsh, float vpd,
                   const CameraState& cam, glmf::mat4* model_cam, glmf::mat4* inverse_view,
                   glmf::mat4* to_volume);

// png.cpp: RGB8 rows top to bottom -> PNG file (throws on I/O failure)
void write_png_rgb8(const std::string& path, int W, int H, const uint8_t* rgb);

}  // namespace vr
