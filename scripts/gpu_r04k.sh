#!/bin/bash
# Ragged key-ownership cost A/B: in-kernel key-run stores and offset stores on / off.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
A=abl
STEPS=10 REPS=2 LIBS="cur= nokcp=$A/nokcp/lib/libmerklekv_hip.so noodst=$A/noodst/lib/libmerklekv_hip.so none=$A/none/lib/libmerklekv_hip.so" \
  bash scripts/gpu_ab_ragged.sh
