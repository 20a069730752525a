set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/split2
mkdir -p $O
for v in 12 10 8; do
  NTT_FS_LOG_N2=$v timeout -k 10 120 python3 tools/exp_split.py 24 1 20 >> $O/check.txt 2>&1 || exit 1
done
NTT_FS_LOG_N2=8 timeout -k 10 120 python3 tools/exp_split.py 24 8 10 >> $O/check.txt 2>&1 || exit 1
NTT_FS_LOG_N2=8 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/p8 -o run --output-format csv -- python3 tools/exp_split.py 24 1 20 > $O/p8.log 2>&1 || exit 1
NTT_FS_LOG_N2=12 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/p12 -o run --output-format csv -- python3 tools/exp_split.py 24 1 20 > $O/p12.log 2>&1 || exit 1
