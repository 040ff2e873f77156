mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_swscale.py tests/test_gpu_pieces.py -x -q --timeout 240 --timeout-method thread > gpurun_out/t_sws.log 2>&1; rc=$?; tail -3 gpurun_out/t_sws.log; [ $rc -eq 0 ] || exit $rc
PARAM=sws_band_group VALUES="1 2 4 8 64" REPS=1 bash tools/ab_param.sh
