#!/bin/bash
# Build the library of git ref $1 (default HEAD) into maddpg_amd/libmaddpg_hip_ref.so
# (a worktree under /tmp; the A/B partner of tools/ab_lib.sh).  Run here, not on the GPU box.
set -e
REF=${1:-HEAD}
WT=/tmp/mdp_ref_wt
rm -rf $WT; git worktree prune
git worktree add -f --detach $WT $REF > /dev/null
make -s -C $WT/maddpg_amd/csrc -j8 > /dev/null
cp $WT/maddpg_amd/libmaddpg_hip.so maddpg_amd/libmaddpg_hip_ref.so
git worktree remove --force $WT
echo "built $REF -> maddpg_amd/libmaddpg_hip_ref.so"
