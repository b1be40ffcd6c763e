set -o pipefail
O=gpurun_out/r02g; mkdir -p $O
export TMPDIR=/tmp
MI_NO_GRAPH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --no-cpu --steps 64 --warmup 8 --prefill 0 > $O/prof_bench.json 2> $O/prof.err || exit $?
find $O/prof -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats.csv \;
rm -rf $O/prof
head -12 $O/kernel_stats.csv | cut -c1-160
MI_NO_GRAPH=1 timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc -o pmc -- python3 -u bench.py --no-cpu --steps 8 --warmup 2 --prefill 0 > $O/pmc_bench.json 2> $O/pmc.err || exit $?
F=$(find $O/pmc -name '*counter_collection.csv' | head -1)
cp "$F" $O/counter_collection.csv
rm -rf $O/pmc
python3 scripts/pmc_traffic.py $O/counter_collection.csv 'gemv_tILi12ELi2ELi16ELi0ELi1E' $O/pmc_ffn.json || python3 -c "
import csv; rows=list(csv.DictReader(open('$O/counter_collection.csv'))); print(rows[0].keys()); print(set(r['Kernel_Name'][:60] for r in rows))"
