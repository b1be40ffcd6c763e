mkdir -p gpurun_out/e4
timeout -k 10 200 ./scripts/exp_gemv2_st 1 > gpurun_out/e4/stamps.txt 2>&1 || exit $?
timeout -k 10 200 ./scripts/exp_gemv2 2 > gpurun_out/e4/chain.txt 2>&1 || exit $?
cat gpurun_out/e4/stamps.txt gpurun_out/e4/chain.txt
