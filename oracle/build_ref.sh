#!/usr/bin/env bash
# Builds oracle/_ref/glm_probe from oracle/ref_glm_probe.cpp against the reference's OWN vendored
# glm 0.9.8.5 (header-only), compiled from where it lies under /root/reference.  Nothing from the
# reference is copied.  The reference's hot-path classes themselves (Octree.cu, BinaryLoader.cu,
# TransferFunction.cu, kernel.cu) are NOT buildable here: they include cuda_runtime.h,
# device_launch_parameters.h, glad/glad.h and GLFW/glfw3.h, which this image lacks, and
# Material.h:31 / TransferFunction.h:36 use MSVC-only syntax.  See DESIGN.md.
set -euo pipefail
HERE="$(cd "$(dirname "$0")" && pwd)"
REF="${VR_REFERENCE:-/root/reference}"
if [ ! -f "$REF/glm/glm.hpp" ]; then echo "build_ref: $REF/glm absent; skipping" >&2; exit 0; fi
mkdir -p "$HERE/_ref"
g++ -O2 -std=c++17 -ffp-contract=off -fno-fast-math -w -I"$REF" "$HERE/ref_glm_probe.cpp" -o "$HERE/_ref/glm_probe"
echo "built $HERE/_ref/glm_probe"
