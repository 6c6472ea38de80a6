# Build a variant of libtfusion_hip.so with extra defines into tools/_build/NAME/ (for A/B runs
# through TFUSION_HIP_LIB, tools/gpu_ab_lib.sh).   bash tools/build_variant.sh NAME -DX=1 ...
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
O=$R/tools/_build/$NAME
mkdir -p $O
cd $R/topfusion_amd/csrc
FL="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero"
objs=""
for f in tf_preproc tf_icp tf_scene tf_render tf_capi tf_imgproc tf_swap tf_fuse; do
  /opt/rocm/bin/hipcc $FL "$@" -c $f.hip -o $O/$f.o &
  objs="$objs $O/$f.o"
done
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -Wl,-z,defs -o $O/libtfusion_hip.so $objs
rm -f $objs
echo "built $O/libtfusion_hip.so"
