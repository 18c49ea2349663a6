# Per-kernel register / occupancy / spill summary of one HIP source (compile-time remarks).
# usage: bash scripts/kres.sh csrc/ctrl.hip [extra hipcc flags]
SRC=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -mcode-object-version=5 -Icsrc "$@" -c $SRC \
  -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 | sed -n 's/.*remark: *//p' | \
  awk '/Function Name/{if(n)print line; line=$3; n=1; next} /VGPRs:|AGPRs:|Occupancy|VGPRs Spill|LDS Size/{gsub(/ \[-Rpass.*/,""); line=line" | "$0} END{print line}' | \
  c++filt | sed 's/(mb::[A-Za-z]*)//'
