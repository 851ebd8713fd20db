#!/bin/bash
# Round 4: quiet-step skips of the clamp, the NULL list and the wr stats: the
# -m gpu suite, smoke and the driver's bench line.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_r4_final_a.sh ${1:-r4l}
