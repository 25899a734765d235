# round-4 call w: STRICT row reverse with two pairs per lane (variant rp2s): FWT parity, cfg4 A/B
mkdir -p gpurun_out/w
JWAVE_HIP_LIB=$PWD/jwave-pro_amd/ab/libjwave_hip_rp2s.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_fwt_gpu.py tests/test_wpt_gpu.py > gpurun_out/w/pytest_rp2s.log 2>&1; rc=$?; tail -1 gpurun_out/w/pytest_rp2s.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_fwt_libs.sh w rp2s
