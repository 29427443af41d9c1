set -o pipefail
O=gpurun_out/r05c; mkdir -p $O
for sh in "16 512 512 128 128 1 1" "16 512 512 128 128 0 1" "16 256 256 256 256 1 1" "16 128 128 512 512 1 1"; do
  timeout -k 5 60 tools/halo_stamps_cur $sh >> $O/stamps.jsonl 2>> $O/err.txt || { echo "stamps failed"; tail $O/err.txt; exit 3; }
  HALO4=1 timeout -k 5 60 tools/halo_stamps_cur $sh >> $O/stamps_h4.jsonl 2>> $O/err.txt || { echo "stamps h4 failed"; exit 3; }
  H256=1 timeout -k 5 60 tools/halo_stamps_cur $sh >> $O/stamps_h256.jsonl 2>> $O/err.txt || { echo "stamps h256 failed"; exit 3; }
done
cat $O/stamps.jsonl $O/stamps_h4.jsonl $O/stamps_h256.jsonl
