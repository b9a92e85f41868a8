set -o pipefail
cd /root/repo && mkdir -p gpurun_out/r04h
timeout -k 10 60 ./profiles/r04/mb_r64 > gpurun_out/r04h/mb_r64.txt 2>&1 || exit 1
bash profiles/r04/prof_wl.sh r04h 'estep_config3 estep estep_demo1_jt' tests/test_gpu_jtree.py tests/test_gpu_estep.py
