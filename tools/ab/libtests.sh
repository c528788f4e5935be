#!/bin/bash
# Run a pytest -m gpu selection against several library builds (each copied over the product in
# turn, the product restored at the end); a test FAILURE (rc 1) moves on to the next build, any
# other exit (fault, abort, time limit) stops the script there.
#   K="ctu or cfg4" bash tools/ab/libtests.sh product tools/_ab/libnanohevc_m0.so ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
P=nano-hevc_amd/nano_hevc/libnanohevc.so
cp $P /tmp/nh_product.so
rc_all=0
for lib in "$@"; do
  name=$(basename $lib .so)
  [ "$lib" != product ] && cp "$lib" $P
  timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread --maxfail=${MAXFAIL:-4} \
    tests -m gpu -k "${K:?set K}" > gpurun_out/libtests_${TAG:-x}_$name.log 2>&1
  rc=$?
  cp /tmp/nh_product.so $P
  echo "== $name rc=$rc: $(tail -1 gpurun_out/libtests_${TAG:-x}_$name.log)"
  grep -E "^FAILED" gpurun_out/libtests_${TAG:-x}_$name.log | head -8
  [ $rc -gt 1 ] && exit $rc
done
exit 0
