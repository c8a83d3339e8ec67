mkdir -p gpurun_out
timeout -k 10 60 ./tools/microbench/mfma_i8_layout > gpurun_out/mfma_layout.txt 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "kernel or many_sketches or join or scale" > gpurun_out/gputest3.log 2>&1
