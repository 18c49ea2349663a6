# Ablation builds of the CBF training kernel (experiment macros CBF_X_* in csrc/cbf.hip): each
# variant = the regular objects with cbf.o replaced, linked to build/variants/<name>/_C.so.
# usage: bash scripts/build_cbf_variants.sh NAME:FLAGS ...   (run python csrc/build.py first)
set -e
R=$(cd $(dirname $0)/.. && pwd)
B=$R/build/csrc
ARCH=gfx950
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  out=$R/build/variants/$name
  mkdir -p $out
  /opt/rocm/bin/hipcc --offload-arch=$ARCH -O3 -fPIC -std=c++17 -mcode-object-version=5 -Wno-unused-result \
    -Wno-unused-variable -I$R/csrc $flags -c $R/csrc/cbf.hip -o $out/cbf.o
  objs=$(ls $B/*.o | grep -v -e '/cbf.o$' -e '/host_')
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=$ARCH $objs $out/cbf.o -o $out/_C.so \
    -Wl,-rpath,$(python -c 'import torch,os;print(os.path.join(os.path.dirname(torch.__file__),"lib"))') -Wl,-rpath,/opt/rocm/lib
  echo "built $out/_C.so ($flags)"
done
