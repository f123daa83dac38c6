#!/bin/bash
# Build the current tree's library with extra compile flags into
# maddpg_amd/libmaddpg_hip_<name>.so (the A/B partner of tools/ab_lib.sh):
#   bash tools/build_variant.sh wt -DMDP_NT_SLAB=2
# Timing-only experiments (-DMDP_EXP_<NAME>: TPRE, R32, BF6, ONE_TACT,
# NO_CRITQ, NOLOAD, NOMFMA, SLAB_NONE, SLAB_HALF, NOLOAD_R, DW_NONE) are not in the product sources: their code
# is tools/variants/mdp_exp.patch, applied to the scratch copy here whenever a
# -DMDP_EXP_ flag is given (tools/variants/strip_exp.py made it).
# Run here, not on the GPU box.
set -e
NAME=$1; shift
D=/tmp/mdp_variant_$NAME
rm -rf $D; mkdir -p $D
mkdir -p $D/maddpg_amd $D/include $D/tools; cp -r maddpg_amd/csrc $D/maddpg_amd/csrc; cp include/*.h $D/include/; cp tools/check_scratch.py $D/tools/
rm -rf $D/maddpg_amd/csrc/build
case " $* " in
  *-DMDP_EXP_*) (cd $D/maddpg_amd/csrc && patch -p1 -s < "$OLDPWD/tools/variants/mdp_exp.patch")
                echo "applied tools/variants/mdp_exp.patch" ;;
esac
make -s -C $D/maddpg_amd/csrc -j8 CXXFLAGS="-O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -Wall -Wno-unused-function $*" OUT=$D/lib.so HDR= $D/lib.so > /dev/null
cp $D/lib.so maddpg_amd/libmaddpg_hip_$NAME.so
rm -rf $D
echo "built variant $NAME ($*) -> maddpg_amd/libmaddpg_hip_$NAME.so"
