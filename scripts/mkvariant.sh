#!/bin/bash
# A/B variant library: copies merklekv_amd/csrc to ab/<name>/src, applies the python patch file (reads
# and rewrites files in the current directory), builds ab/<name>/lib/libmerklekv_hip.so. Load it with
# MKV_LIB_PATH=ab/<name>/lib/libmerklekv_hip.so. ab/ is git-ignored (the .so still travels to the GPU box).
set -e
cd "$(dirname "$0")/.."
name=$1; patch=$2
rm -rf ab/$name && mkdir -p ab/$name && cp -r merklekv_amd/csrc ab/$name/src
ln -sfn ../include ab/include
if [ -n "$patch" ]; then (p=$(readlink -f "$patch"); cd ab/$name/src && python3 "$p"); fi
make -C ab/$name/src -j8 > ab/$name/build.log 2>&1 || { tail -20 ab/$name/build.log; exit 1; }
ls -la ab/$name/lib/libmerklekv_hip.so
