set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/tiling_ab.py --stripes 1 2>&1 | grep -v Warn
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tiling_prof -o run -- python3 tools/tiling_ab.py --stripes 1 --rounds 1 > gpurun_out/tiling_prof.log 2>&1 || exit 1
cut -d, -f1-5 gpurun_out/tiling_prof/run_kernel_stats.csv | head -5
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/tiling_prof/run_kernel_trace.csv')))
f=[r for r in rows if 'fold' in r['Kernel_Name']]
for r in f: print('fold', r.get('Grid_Size_X', r.get('Grid_Size','?')), (int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e6, 'ms')
PY
