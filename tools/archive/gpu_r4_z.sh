#!/bin/bash
# Round 4: PPO profiles (f32 / bf16 kernel splits + MFMA-busy PMC) at HEAD.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_ppo_prof.sh
