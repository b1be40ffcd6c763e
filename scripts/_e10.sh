mkdir -p gpurun_out/e10
MI_GEMV_ORDER=2 MI_GEMV_PRE=0 MI_ENGINE_LIB=stamps timeout -k 10 300 python -u scripts/timeline.py llama2-7b-q4_k_m 64 > gpurun_out/e10/timeline.txt 2>&1 || exit $?
grep -E "launch +[0-9]+:" gpurun_out/e10/timeline.txt
