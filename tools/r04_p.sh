# round-4 call p: product MODWT GPU tests (ring rotation on), then the MODWT benches against
# builds of the fast MODWT kernels with other AMDGPU scheduling strategies
mkdir -p gpurun_out/p
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_modwt_gpu.py tests/test_modwt_strict_gpu.py tests/test_jni_glue_gpu.py tests/test_host_pipeline_gpu.py -k "not default_geometry and not auto_2_25" > gpurun_out/p/pytest_modwt.log 2>&1; rc=$?; tail -2 gpurun_out/p/pytest_modwt.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_modwt_libs.sh p mmc iilp milp
