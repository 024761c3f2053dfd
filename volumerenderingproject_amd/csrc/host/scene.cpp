// scene.cpp -- host model of the render path (see scene.h for the reference map).
#include "scene.h"

#include <cmath>
#include <cstring>
#include <fstream>

#include "../../../include/vr_api.h"

#pragma clang fp contract(off)

namespace vr {

// ============================================ NiftiFile =====================================

namespace {
template <class T> T bswap(T v) {
    unsigned char b[sizeof(T)];
    std::memcpy(b, &v, sizeof(T));
    for (size_t i = 0; i < sizeof(T) / 2; ++i) std::swap(b[i], b[sizeof(T) - 1 - i]);
    std::memcpy(&v, b, sizeof(T));
    return v;
}
template <class T> T rd(const unsigned char* p, bool sw) {
    T v;
    std::memcpy(&v, p, sizeof(T));
    return sw ? bswap(v) : v;
}
}  // namespace

NiftiFile::NiftiFile(const std::string& filename) {
    std::ifstream file(filename, std::ios::in | std::ios::binary | std::ios::ate);
    if (!file.is_open()) throw Error(VR_EIO, "NiftiFile: unable to open " + filename);
    const std::streamoff size = file.tellg();
    unsigned char h[540];
    std::memset(h, 0, sizeof h);
    file.seekg(0, std::ios::beg);
    file.read(reinterpret_cast<char*>(h), size < 540 ? size : 540);
    if (size < 348) throw Error(VR_EIO, "NiftiFile: file too short for a NIfTI header: " + filename);
    int32_t sh = rd<int32_t>(h, false);
    bool sw = false;
    if (sh != 540 && sh != 348) {
        sh = rd<int32_t>(h, true);
        sw = true;
        if (sh != 540 && sh != 348)
            throw Error(VR_EIO, "NiftiFile: not a NIfTI-1/2 file (sizeof_hdr) " + filename);
    }
    header.sizeof_hdr = sh;
    if (sh == 540) {   // nifti2.h:59-98 (packed offsets)
        header.datatype = rd<int16_t>(h + 12, sw);
        header.bitpix = rd<int16_t>(h + 14, sw);
        for (int i = 0; i < 8; ++i) header.dim[i] = rd<int64_t>(h + 16 + 8 * i, sw);
        for (int i = 0; i < 8; ++i) header.pixdim[i] = rd<double>(h + 104 + 8 * i, sw);
        header.vox_offset = rd<int64_t>(h + 168, sw);
        header.scl_slope = rd<double>(h + 176, sw);
        header.scl_inter = rd<double>(h + 184, sw);
        header.cal_max = rd<double>(h + 192, sw);
        header.cal_min = rd<double>(h + 200, sw);
    } else {           // NIfTI-1 (nifti1.h, 348-byte header)
        for (int i = 0; i < 8; ++i) header.dim[i] = rd<int16_t>(h + 40 + 2 * i, sw);
        header.datatype = rd<int16_t>(h + 70, sw);
        header.bitpix = rd<int16_t>(h + 72, sw);
        for (int i = 0; i < 8; ++i) header.pixdim[i] = rd<float>(h + 76 + 4 * i, sw);
        // a float field: NaN, infinite or out-of-range offsets are refused before the conversion
        // (converting them to an integer is undefined; found by the UBSan fuzz, tests/test_sanitize.py)
        const float vo = rd<float>(h + 108, sw);
        if (!(vo >= 0.0f && vo < 9.0e18f)) throw Error(VR_EIO, "NiftiFile: bad vox_offset in " + filename);
        header.vox_offset = (int64_t)vo;
        header.scl_slope = rd<float>(h + 112, sw);
        header.scl_inter = rd<float>(h + 116, sw);
        header.cal_max = rd<float>(h + 124, sw);
        header.cal_min = rd<float>(h + 128, sw);
    }
    if (header.dim[0] < 3 || header.dim[1] <= 0 || header.dim[2] <= 0 || header.dim[3] <= 0)
        throw Error(VR_EFORMAT, "NiftiFile: need a 3-D volume");
    for (int i = 4; i <= header.dim[0] && i < 8; ++i)
        if (header.dim[i] > 1) throw Error(VR_EFORMAT, "NiftiFile: 4-D and higher volumes are not supported");
    // untrusted int64 dims (NIfTI-2): each within the int32 voxel index of a row and the product
    // checked before any multiplication can wrap (a wrapped count would pass the size check below
    // while the kernels index with the real dims)
    constexpr int64_t kMaxDim = ((int64_t)1 << 31) - 1, kMaxVoxels = (int64_t)1 << 40;
    for (int a = 1; a <= 3; ++a)
        if (header.dim[a] > kMaxDim) throw Error(VR_ERANGE, "NiftiFile: dimension too large in " + filename);
    if (header.dim[1] > kMaxVoxels / header.dim[2] || header.dim[1] * header.dim[2] > kMaxVoxels / header.dim[3])
        throw Error(VR_ERANGE, "NiftiFile: volume too large in " + filename);
    const int64_t n = header.dim[1] * header.dim[2] * header.dim[3];
    int bytes = 0;
    switch (header.datatype) {
        case 2: case 256: bytes = 1; break;        // uint8, int8
        case 4: case 512: bytes = 2; break;        // int16, uint16
        case 8: case 768: case 16: bytes = 4; break;   // int32, uint32, float32
        case 64: bytes = 8; break;                 // float64
        default: throw Error(VR_EFORMAT, "NiftiFile: unsupported datatype " + std::to_string(header.datatype));
    }
    if (header.vox_offset < 0 || header.vox_offset > size || n > (size - header.vox_offset) / bytes)
        throw Error(VR_EIO, "NiftiFile: truncated voxel data in " + filename);
    std::vector<unsigned char> raw((size_t)(n * bytes));
    file.seekg(header.vox_offset, std::ios::beg);
    file.read(reinterpret_cast<char*>(raw.data()), (std::streamsize)raw.size());
    if (!file) throw Error(VR_EIO, "NiftiFile: read failed " + filename);
    volume.resize((size_t)n);
    const unsigned char* p = raw.data();
    for (int64_t i = 0; i < n; ++i, p += bytes) {
        float v = 0;
        switch (header.datatype) {
            case 2: v = (float)p[0]; break;
            case 256: v = (float)(int8_t)p[0]; break;
            case 4: v = (float)rd<int16_t>(p, sw); break;
            case 512: v = (float)rd<uint16_t>(p, sw); break;
            case 8: v = (float)rd<int32_t>(p, sw); break;
            case 768: v = (float)rd<uint32_t>(p, sw); break;
            case 16: v = rd<float>(p, sw); break;
            case 64: v = (float)rd<double>(p, sw); break;
        }
        volume[(size_t)i] = v;
    }
    finish();
}

NiftiFile::NiftiFile(std::vector<float> vol, int64_t d1, int64_t d2, int64_t d3, double cal_max) {
    if (d1 <= 0 || d2 <= 0 || d3 <= 0 || (int64_t)vol.size() != d1 * d2 * d3)
        throw Error(VR_EINVAL, "NiftiFile: volume size does not match dims");
    header.dim[1] = d1; header.dim[2] = d2; header.dim[3] = d3;
    header.cal_max = cal_max;
    volume = std::move(vol);
    finish();
}

void NiftiFile::finish() {
    longest_dimension = 0;
    for (int i = 0; i < 3; ++i)
        if (header.dim[i + 1] > longest_dimension) longest_dimension = (int)header.dim[i + 1];
    totaldim = header.dim[1] * header.dim[2] * header.dim[3];
}

// ============================================ Material / TF ==================================

namespace Material {
Material getMaterialFromID(MaterialId id) {   // Material.cpp:6-67
    switch (id) {
        case red: return {"RED", {1.0f, 0.0f, 0.0f, 1.0f}, 0.0};
        case green: return {"GREEN", {0.0f, 1.0f, 0.0f, 1.0f}, 0.0};
        case blue: return {"BLUE", {0.0f, 0.0f, 1.0f, 1.0f}, 0.0};
        case glass: return {"GLASS", {0.2f, 0.2f, 0.2f, 0.1f}, 0.0};
        case muscle: return {"MUSCLE", {124.0f / 255.0f, 9.0f / 255.0f, 42.0f / 255.0f, 0.3f}, 0.0};
        case empty: return {"EMPTY", {0.0f, 0.0f, 0.0f, 0.0f}, 0.0};
        case bone: return {"BONE", {241.0f / 255.0f, 218.0f / 255.0f, 202.0f / 255.0f, 0.3f}, 0.0};
        case brain: return {"BRAIN", {223.0f / 255.0f, 155.0f / 255.0f, 141.0f / 255.0f, 0.7f}, 0.0};
        case brain_stem: return {"BRAIN_STEM", {241.0f / 255.0f, 218.0f / 255.0f, 202.0f / 255.0f, 0.9f}, 0.0};
        case cerebelum: return {"CEREBELUM", {241.0f / 255.0f, 218.0f / 255.0f, 202.0f / 255.0f, 0.9f}, 0.0};
        case cerebrospinal_fluid:
            return {"CEREBROSPINAL_FLUID", {241.0f / 255.0f, 218.0f / 255.0f, 202.0f / 255.0f, 0.9f}, 0.0};
        case eye: return {"EYE", {241.0f / 255.0f, 218.0f / 255.0f, 202.0f / 255.0f, 0.9f}, 0.0};
        default: return {"DEFAULT", {1.0f, 0.0f, 1.0f, 0.1f}, 0.0};
    }
}
}  // namespace Material

TransferFunction::TransferFunction() {   // TransferFunction.cu:19-23
    using namespace Material;
    material_intervals = {
        {getMaterialFromID(empty), 0.0f, 1.0f},
        {getMaterialFromID(bone), 30.0f / 255.0f, 80.0f / 255.0f},
        {getMaterialFromID(muscle), 140.0f / 255.0f, 160.0f / 255.0f},
        {getMaterialFromID(brain), 105.0f / 255.0f, 120.0f / 255.0f},
    };
}

TransferFunction::TransferFunction(std::vector<MatInterval> iv) : material_intervals(std::move(iv)) {
    if (material_intervals.empty()) throw Error(VR_EINVAL, "TransferFunction: no intervals");
}

int TransferFunction::getMaterialIndex(float value) const {
    int r = 0;
    for (int i = 0; i < size(); ++i)
        if (value >= material_intervals[i].lower_bound && value <= material_intervals[i].higher_bound) r = i;
    return r;
}

// ============================================ OctreeHandler ==================================

void OctreeHandler::build(int64_t d1, int64_t d2, int64_t d3) {
    const int64_t d[3] = {d1, d2, d3};
    longest_dimension = 0;
    for (int i = 0; i < 3; ++i)
        if (longest_dimension < (uint32_t)d[i]) longest_dimension = (uint32_t)d[i];
    maximum_depth = 0;
    while (std::pow(2, maximum_depth) < longest_dimension) maximum_depth++;   // Octree.cu:40-41
    if (maximum_depth > 24) throw Error(VR_ERANGE, "OctreeHandler: volume too large");
    number_of_nodes = 0;
    for (uint32_t p = 0; p <= maximum_depth; ++p) number_of_nodes += (uint64_t)1 << (3 * p);
    nleaf = 1 << maximum_depth;
    maps.assign((size_t)3 * nleaf, -1);
    const float L = (float)longest_dimension;   // glm::scale by vec3(L) (Octree.cu:86)
    const float hL = (float)longest_dimension / 2.0f;
    const float leaves = (float)nleaf;
    for (int a = 0; a < 3; ++a) {
        const float h = (float)d[a] / 2.0f;
        const float lo = hL - h, hi = hL + h;   // Octree.cu:92-94
        leaf_lo[a] = nleaf; leaf_hi[a] = -1;
        for (int i = 0; i < nleaf; ++i) {
            const float lc = (float)i / leaves;     // createNode's dyadic corner, exact
            const float res = L * lc;               // scaleMatrix * vec4(lc, 1): zeros add exactly
            if (res >= lo && res < hi) {
                int v = (int)((res + h) - hL);      // Octree.cu:97-100
                if (v >= d[a]) v = (int)d[a] - 1;   // unreachable for valid inputs; keeps indices in range
                maps[(size_t)a * nleaf + i] = v;
                if (i < leaf_lo[a]) leaf_lo[a] = i;
                leaf_hi[a] = i;
            }
        }
    }
}

// ============================================ camera ==========================================

void default_screen(int W, int H, int S, float* rsw, float* rsh, float* vpd, float* fc, float* sd) {
    const float view_angle = (float)(M_PI / 4);             // utils.h:54
    const float w = 2 * std::tan(view_angle);               // utils.h:58 (orthographic)
    *rsw = w;
    *rsh = w * (float)(unsigned)H / (float)(unsigned)W;     // utils.h:59
    *vpd = 2.0f;                                            // utils.h:53
    *fc = 0.0f;                                             // utils.h:73
    *sd = (*vpd - *fc) / (float)(unsigned)S;                // utils.h:74
}

CameraState derive_camera(glmf::vec3 pos, glmf::vec3 up, float rsw, float rsh) {
    using namespace glmf;
    const mat4 rt = mul(identity(), identity());
    const vec4 p4 = mul(rt, v4(pos.x, pos.y, pos.z, 1.0f));
    CameraState c;
    c.pos = v3(p4.x, p4.y, p4.z);
    c.front = normalize(v3(0.0f, 0.0f, 0.0f) - c.pos);
    c.right = normalize(cross(up, c.front));
    c.up = cross(c.front, c.right);
    c.top_left = (c.pos + (rsw / 2) * (-c.right)) + (c.up * (rsh / 2));
    return c;
}

CameraState derive_camera_conic(glmf::vec3 pos, glmf::vec3 up, float rsw, float rsh, float vpd) {
    using namespace glmf;
    CameraState c = derive_camera(pos, up, rsw, rsh);
    // utils.h:93-97 (conic branch of updateTopLeftCorner)
    c.top_left = ((c.pos + (vpd * c.front)) + (rsw / 2) * (-c.right)) + (c.up * (rsh / 2));
    return c;
}

CameraState default_camera(int W, int H) {
    using namespace glmf;
    float rsw, rsh, vpd, fc, sd;
    default_screen(W, H, 1, &rsw, &rsh, &vpd, &fc, &sd);
    const vec3 pos = v3(0.0f, 0.0f, 1.0f);                       // utils.h:41-46
    const vec3 front = normalize(v3(0.0f, 0.0f, 0.0f) - pos);
    const vec3 up0 = v3(0.0f, 1.0f, 0.0f);
    const vec3 right = normalize(cross(front, up0));
    const vec3 up = normalize(cross(right, front));
    return derive_camera(pos, up, rsw, rsh);
}

CameraState reset_camera() {   // utils.h:77-81
    CameraState c;
    c.pos = {0.456607f, 0.693644f, (float)-0.55711};
    c.front = {-0.456606f, -0.693643f, 0.557109f};
    c.right = {-0.19427f, -0.533349f, -0.823285f};
    c.up = {0.868199f, -0.484147f, 0.108777f};
    c.top_left = {1.51908f, 0.742847f, 0.374952f};
    return c;
}

void test_matrices(int64_t d1, int64_t d2, int64_t d3, int W, int H, int S, float rsw, float rsh, float vpd,
                   const CameraState& cam, glmf::mat4* model_cam, glmf::mat4* inverse_view,
                   glmf::mat4* to_volume) {
    using namespace glmf;
    mat4 mc = translate(identity(), v3(-rsw / 2.0f, -rsh / 2.0f, 0.0f));   // kernel.cu:1177-1190
    mc = scale(mc, v3(rsw / (float)(unsigned)W, rsh / (float)(unsigned)H, -vpd / (float)(unsigned)S));
    mat4 view = inverse(lookAt(cam.pos, v3(0.0f, 0.0f, 0.0f), cam.up));     // kernel.cu:1194-1195
    int64_t Ld = d1 > d2 ? d1 : d2;
    if (d3 > Ld) Ld = d3;
    const int L = (int)Ld;
    mat4 tv = identity();                                                    // kernel.cu:1200-1216
    const mat4 t1 = translate(identity(), v3(0.5f, 0.5f, 0.5f));
    const mat4 sc = scale(identity(), v3((float)L, (float)L, (float)L));
    const mat4 t2 = translate(identity(), v3((float)d1 / 2.0f - (float)L / 2.0f, (float)d2 / 2.0f - (float)L / 2.0f,
                                             (float)d3 / 2.0f - (float)L / 2.0f));
    tv = mul(t1, tv);
    tv = mul(sc, tv);
    tv = mul(t2, tv);
    *model_cam = mc;
    *inverse_view = view;
    *to_volume = tv;
}

}  // namespace vr
