"""MI355X-native direct-volume ray marcher (drop-in for RodrigoGomesSantos/VolumeRenderingProject's
render path).  The product is libvr.so (HIP kernels for gfx950 + C-ABI, include/vr_api.h); this
package is its Python binding.  See DESIGN.md."""
from .renderer import (VR_FLAG_CONIC, VR_FLAG_ERT, VR_FLAG_ESS, VR_FLAG_SHADE, VR_MODE_TEST, VR_MODE_VRC, Camera,  # noqa: F401
                       Options, RenderParams, VolumeRenderer, VRError, default_camera, default_options,
                       default_params,
                       default_transfer_function, derive_camera, derive_camera_conic, device_count, lib,
                       reset_camera)

__version__ = "0.1.0"
