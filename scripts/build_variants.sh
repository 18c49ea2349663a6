# Ablation / experiment builds of one kernel source: each variant = the regular objects with
# <src>.o replaced by a build with extra flags, linked to build/variants/<name>/_C.so.
# usage: bash scripts/build_variants.sh SRC NAME:FLAGS ...   (SRC = cbf | ctrl | scan | ctrl_x3 |
# cbf_f16 ...: a _x3 / _f16 suffix selects that precision instantiation of the source; run
# python csrc/build.py first). Time them with scripts/micro_cbf.py / micro_step.py --so.
set -e
R=$(cd $(dirname $0)/.. && pwd)
B=$R/build/csrc
ARCH=gfx950
SRC=$1; shift
FILE=${SRC%_x3}; FILE=${FILE%_f16}; PFL=""
case $SRC in *_x3) PFL="-DMB_X3=1";; *_f16) PFL="-DMB_FP16=1";; esac
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  out=$R/build/variants/$name
  mkdir -p $out
  /opt/rocm/bin/hipcc --offload-arch=$ARCH -O3 -fPIC -std=c++17 -mcode-object-version=5 -Wno-unused-result \
    -Wno-unused-variable -I$R/csrc $PFL $flags -c $R/csrc/$FILE.hip -o $out/$SRC.o
  objs=$(ls $B/*.o | grep -v -e "/$SRC.o\$" -e '/host_')
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=$ARCH $objs $out/$SRC.o -o $out/_C.so \
    -Wl,-rpath,$(python -c 'import torch,os;print(os.path.join(os.path.dirname(torch.__file__),"lib"))') -Wl,-rpath,/opt/rocm/lib
  echo "built $out/_C.so ($SRC $flags)"
done
