#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_r04l.sh && bash tools/gpu_r04m.sh
