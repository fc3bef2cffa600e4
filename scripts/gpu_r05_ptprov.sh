#!/bin/bash
# round 5: use_infinite / PT provenance / ptgen scratch tests on the GPU, the phonon-map correlation goldens
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/r05_ptprov
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_ptgen.py tests/test_correlations_golden.py tests/test_gpu_parity.py \
    -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider \
    -k "tls_reference_default or infinite or refuses or driver_generates or ibm or scratch or svd or jacobi or phonon or map_tail or tl_" \
    > $O/pytest_ptprov2.log 2>&1
rc=$?
tail -30 $O/pytest_ptprov2.log
exit $rc
