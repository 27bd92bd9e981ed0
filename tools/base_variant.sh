#!/bin/bash
# tools/base_variant.sh TAG [DEFS] — build the committed HEAD sources as experiment library
# libxrt_hip_TAG.so (for A/B runs against the working tree), then rebuild the working tree.
set -euo pipefail
cd "$(dirname "$0")/.."
git stash -q
trap 'git stash pop -q; make -s -C xraytracer_amd/csrc' EXIT
make -s -C xraytracer_amd/csrc variant TAG=$1 DEFS="${2:-}"
