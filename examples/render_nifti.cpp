// render_nifti -- a C++ host over libvr in the shape of the reference's application
// (myApp.cu main + renderLoop, VRC / TEST branches :877-1052): load a NIfTI volume with NiftiFile,
// take the reference transfer function, build the octree leaf grid, put the volume on the GPU and
// render one frame of the steady default camera (AppData utils.h:41-46 + processInput), saved as
// the reference's window would show it (saveImage, myApp.cu:1942-1956).
//
// usage: render_nifti <volume.nii> <out.png> [width height samples] [vrc|test] [exact|fast] [gpus]
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "vr_api.h"
#include "vr_scene.hpp"

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: %s <volume.nii> <out.png> [W H S] [vrc|test] [exact|fast] [gpus]\n", argv[0]);
        return 2;
    }
    const int W = argc > 5 ? std::atoi(argv[3]) : 300, H = argc > 5 ? std::atoi(argv[4]) : 300,
              S = argc > 5 ? std::atoi(argv[5]) : 300;
    const bool test = argc > 6 && std::strcmp(argv[6], "test") == 0;
    const bool fast = argc > 7 && std::strcmp(argv[7], "fast") == 0;
    const int gpus = argc > 8 ? std::atoi(argv[8]) : 1;
    try {
        vr::NiftiFile nf(argv[1]);                       // BinaryLoader.cu:273-335 (fails hard)
        vr::TransferFunction tf;                         // TransferFunction.cu:8-39
        vr::OctreeHandler oct;                           // Octree.cu:30-53, closed-form leaf grid
        oct.build(nf.header.dim[1], nf.header.dim[2], nf.header.dim[3]);
        std::printf("volume %lldx%lldx%lld cal_max %g, octree depth %u (%llu nodes in the reference's tree)\n",
                    (long long)nf.header.dim[1], (long long)nf.header.dim[2], (long long)nf.header.dim[3],
                    nf.header.cal_max, oct.maximum_depth, (unsigned long long)oct.number_of_nodes);
        std::vector<int32_t> devices(gpus > 0 ? gpus : 1);
        for (size_t i = 0; i < devices.size(); ++i) devices[i] = (int32_t)i;
        vr::VolumeRenderer r = gpus > 1 ? vr::VolumeRenderer(nf, tf, devices) : vr::VolumeRenderer(nf, tf, 0);
        vr_params p;
        vr_params_default(W, H, S, &p);                  // AppData, utils.h:36-74
        p.mode = test ? VR_MODE_TEST : VR_MODE_VRC;
        p.flags = fast ? (VR_FLAG_ESS | VR_FLAG_ERT) : 0;
        vr_camera cam;
        vr_camera_default(W, H, &cam);                   // utils.h:41-46 + processInput
        r.render_png(p, cam, argv[2], test ? VR_ORIENT_TEST_DISPLAY : VR_ORIENT_VRC_DISPLAY);
        const std::vector<float> frame = r.render(p, cam);
        double sum = 0;
        for (float v : frame) sum += v;
        std::printf("rendered %dx%dx%d %s %s on %d GPU(s): %s, channel sum %.6f\n", W, H, S, test ? "TEST" : "VRC",
                    fast ? "ESS+ERT" : "exact", gpus, argv[2], sum);
    } catch (const vr::Error& e) {
        std::fprintf(stderr, "render_nifti: %s (status %d)\n", e.what(), e.code);
        return 1;
    }
    return 0;
}
