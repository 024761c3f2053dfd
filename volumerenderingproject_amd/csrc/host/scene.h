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

#include "../../../include/vr_scene.hpp"
#include "glm_float.h"

namespace vr {

// (NiftiFile, Material, TransferFunction, OctreeHandler: the public classes, include/vr_scene.hpp)

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
