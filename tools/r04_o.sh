# round-4 call o: wave2 inverse with rotated level-6 rings (variant "rot"): MODWT parity, A/B
mkdir -p gpurun_out/o
JWAVE_HIP_LIB=$PWD/jwave-pro_amd/ab/libjwave_hip_rot.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_modwt_gpu.py > gpurun_out/o/pytest_rot.log 2>&1; rc=$?; tail -2 gpurun_out/o/pytest_rot.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_modwt_libs.sh o rot
