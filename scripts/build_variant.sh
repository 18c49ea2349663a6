#!/bin/bash
# Alternative build of the extension with some kernel files recompiled under extra flags, for A/B
# runs on the GPU box (MACBF_EXT=alt_so/NAME/_C.so, or scripts/*.py --so PATH). Usage:
#   scripts/build_variant.sh NAME KERNEL[,KERNEL...] "EXTRA FLAGS"
#   e.g.  v1 cbf_x3 "-DCBF16_SCHED_FWD=1"      k16wg1 cbf,ctrl,cbf_f16,ctrl_f16 "-DCBF16_WGPC=1"
# -> alt_so/NAME/_C.so (git-ignored, travels with the gpurun snapshot)
set -e
cd "$(dirname "$0")/.."
NAME=$1; KS=$2; FL=$3
B=build/csrc; O=alt_so/$NAME; mkdir -p $O
IFS=',' read -ra KL <<< "$KS"
for K in "${KL[@]}"; do
  case $K in *_x3) SRC=${K%_x3}; KD=-DMB_X3=1;; *_f16) SRC=${K%_f16}; KD=-DMB_FP16=1;; *) SRC=$K; KD=;; esac
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -mcode-object-version=5 -Wno-unused-result \
    -Wno-unused-variable -Icsrc $KD $FL -c csrc/$SRC.hip -o $O/$K.o &
  PIDS="$PIDS $!"
done
for p in $PIDS; do wait $p; done      # set -e: a failed compile stops the script
OBJS=""
for o in scan scenario ctrl ctrl_f16 ctrl_x3 cbf cbf_f16 cbf_x3 dedup graph optim bindings runtime; do
  if [[ ",$KS," == *",$o,"* ]]; then OBJS="$OBJS $O/$o.o"; else OBJS="$OBJS $B/$o.o"; fi
done
TL=$(python3 -c "import os,importlib.util as u;print(os.path.join(os.path.dirname(u.find_spec('torch').origin),'lib'))")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -Wl,-rpath,$TL -Wl,-rpath,/opt/rocm/lib $OBJS -o $O/_C.so
echo $O/_C.so
