set -u
mkdir -p gpurun_out/cfg
timeout -k 10 400 python -u bench.py --n 1024 --no-hbm-probe > gpurun_out/cfg/c1.log 2>&1 && tail -1 gpurun_out/cfg/c1.log | cut -c1-150 && \
timeout -k 10 600 python -u bench.py --n 32768 --classes 3 --no-hbm-probe --no-cpu-as-written > gpurun_out/cfg/c3.log 2>&1 && tail -1 gpurun_out/cfg/c3.log | cut -c1-150 && \
timeout -k 10 400 python -u bench.py --n 4096 --features 2048 --no-hbm-probe --no-cpu-as-written > gpurun_out/cfg/f2048.log 2>&1 && tail -1 gpurun_out/cfg/f2048.log | cut -c1-150
