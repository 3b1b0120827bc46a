# SuperPoint forward kernel summary with and without the 64 -> 64 matrix-core convolutions
set -e
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/r04n
for M in c64 no_c64; do
  E=""; [ $M = no_c64 ] && E="FD_SP_NO_C64=1"
  env $E timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04n/$M -o run -- python3 tools/sp_layer_prof.py > gpurun_out/r04n/$M.log 2>&1
  f=$(find gpurun_out/r04n/$M -name '*kernel_stats.csv' | head -1)
  python3 -c "
import csv
rows=sorted(csv.DictReader(open('$f')), key=lambda r: -float(r['TotalDurationNs']))
for r in rows[:12]: print('$M', r['Name'][:90], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us avg')
"
  rm -rf gpurun_out/r04n/$M
done
FD_LIB_PATH=$GRAFT_REPO_ROOT/abvar/c64unroll.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04n/unr -o run -- python3 tools/sp_layer_prof.py > gpurun_out/r04n/unr.log 2>&1
f=$(find gpurun_out/r04n/unr -name '*kernel_stats.csv' | head -1)
python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'conv3x3' in r['Name']: print('unrolled', r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us avg')
"
rm -rf gpurun_out/r04n/unr
