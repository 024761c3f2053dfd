#!/usr/bin/env bash
# Builds A/B variants of libvr.so into build_ab/<name>.so (own object dir each), for
# tools/ab_libs.sh on the GPU box.  usage: tools/build_ab.sh <name> "<-D flags>" [<name> "<flags>" ...]
set -e
cd "$(dirname "$0")/.."
mkdir -p build_ab
while [ $# -ge 2 ]; do
  make -s -j8 -C volumerenderingproject_amd/csrc BDIR="../../build_ab/obj_$1" OUT="../../build_ab/$1.so" EXTRA="$2"
  shift 2
done
ls -la build_ab/*.so
