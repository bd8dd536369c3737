#!/bin/bash
# Host-side AddressSanitizer pass (CPU only -- GPU sanitizers are not available on
# the MI355X pool): libhedgeenv and librbergomi rebuilt with the HOST code instrumented
# (-Xarch_host -fsanitize=address; the gfx950 device code is compiled as usual), then the
# CPU suites that drive every host entry point -- SeedSequence / PCG64 seeding, the host
# RNG / division / exp / Box-Muller builds, he_config / he_create validation, the
# rBergomi estimator and its DFA Hurst fit -- run against them:
#     bash tools/asan/run.sh            (about 5 minutes; log in tools/asan/last.log)
# The ASan runtime is put first on LD_PRELOAD for the pytest process only (ahead of
# whatever the environment already preloads, which stays); leaks are not checked (the
# Python interpreter and torch keep their allocations to exit).
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd); cd $R
O=$R/tools/asan; LOG=$O/last.log
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
ASAN_RT=$(/opt/rocm/lib/llvm/bin/clang -print-file-name=libclang_rt.asan-x86_64.so)
[ -f "$ASAN_RT" ] || ASAN_RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
COMMON="--offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -shared -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt \
 -fno-gpu-flush-denormals-to-zero -Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer -shared-libsan"
S=cantorrl_amd/csrc
{
  echo "[$(date +%T)] build (host ASan): $ASAN_RT"
  $HIPCC $COMMON -o $O/libhedgeenv_asan.so $S/hedge_env.hip $S/vecnorm.hip $S/analytics.hip || exit 1
  $HIPCC $COMMON -o $O/librbergomi_asan.so $S/rbergomi.hip || exit 1
  # positive control: the same build line and runtime set-up must catch a heap overflow
  printf '#include <hip/hip_runtime.h>\n#include <stdlib.h>\nextern "C" int asan_canary(int k) { int* a = (int*)malloc(4 * sizeof(int)); a[k] = 1; int r = a[0]; free(a); return r; }\n' > $O/canary.hip
  $HIPCC $COMMON -o $O/libcanary.so $O/canary.hip || exit 1
  if ASAN_OPTIONS=detect_leaks=0:verify_asan_link_order=0 LD_PRELOAD="$ASAN_RT${LD_PRELOAD:+:$LD_PRELOAD}" \
     python -c "import ctypes; ctypes.CDLL('$O/libcanary.so').asan_canary(4)" > $O/canary.out 2>&1; then
    echo "positive control NOT caught: ASan is not active"; exit 1
  fi
  grep -m1 -o "AddressSanitizer: heap-buffer-overflow" $O/canary.out && echo "positive control caught (heap-buffer-overflow)"
  echo "[$(date +%T)] pytest tests/test_lib_cpu.py tests/test_rbergomi_cpu.py under ASan"
  CANTORRL_HEDGEENV_LIB=$O/libhedgeenv_asan.so CANTORRL_RBERGOMI_LIB=$O/librbergomi_asan.so \
  ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1:verify_asan_link_order=0 \
  LD_PRELOAD="$ASAN_RT${LD_PRELOAD:+:$LD_PRELOAD}" \
    python -m pytest tests/test_lib_cpu.py tests/test_rbergomi_cpu.py -q -p no:cacheprovider
  rc=$?
  echo "[$(date +%T)] exit $rc"
  exit $rc
} 2>&1 | tee $LOG
