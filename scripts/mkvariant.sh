#!/bin/bash
# A/B variant library: copies merklekv_amd/csrc to ab/<name>/src, applies the python patch file (reads
# and rewrites files in the current directory), builds ab/<name>/lib/libmerklekv_hip.so. Load it with
# MKV_LIB_PATH=abl/<name>/lib/libmerklekv_hip.so. abl/ is git-ignored but travels to the GPU box.
set -e
cd "$(dirname "$0")/.."
name=$1; patch=$2
rm -rf abl/$name && mkdir -p abl/$name && cp -r merklekv_amd/csrc abl/$name/src
ln -sfn ../include abl/include
if [ -n "$patch" ]; then (p=$(readlink -f "$patch"); cd abl/$name/src && python3 "$p"); fi
make -C abl/$name/src -j8 > abl/$name/build.log 2>&1 || { tail -20 abl/$name/build.log; exit 1; }
ls -la abl/$name/lib/libmerklekv_hip.so
