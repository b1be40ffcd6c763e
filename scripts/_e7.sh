mkdir -p gpurun_out/e7
timeout -k 10 300 python -u scripts/decode_modes.py > gpurun_out/e7/modes.txt 2>&1 || exit $?
cat gpurun_out/e7/modes.txt
MI_ENGINE_LIB=stamps timeout -k 10 300 python -u scripts/timeline.py llama2-7b-q4_k_m 64 > gpurun_out/e7/timeline.txt 2>&1 || exit $?
sed -n 1,25p gpurun_out/e7/timeline.txt; tail -2 gpurun_out/e7/timeline.txt
