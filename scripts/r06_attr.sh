#!/bin/bash
# r06: the full-depth Mixtral test with its MoE row attribution printed (-s), then the fat-workgroup
# chain experiment (scripts/exp_fat.cpp, mode 2: the 7B step as thin / fat / fat + in-workgroup
# activation launches).
OUT=gpurun_out/${1:-r06_attr}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_gpu_fulldepth.py \
    -k "mixtral" > $OUT/fulldepth_mixtral.log 2>&1
rc=$?; grep -E "attribution|near-tie|median|passed|failed" $OUT/fulldepth_mixtral.log | tail -30; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 ./scripts/exp_fat 2 > $OUT/exp_fat.txt 2>&1 || { echo "exp rc=$?"; tail $OUT/exp_fat.txt; exit 1; }
cat $OUT/exp_fat.txt
