set -o pipefail
OUT=gpurun_out/r04z; mkdir -p $OUT
for rep in 1 2; do for v in prev 2_1; do
  timeout -k 10 120 python3 -u tools/nf_ab.py --lib tools/ab_libs/libmmb_nf_$v.so >> $OUT/ab.txt 2>>$OUT/ab.err || exit 1
  timeout -k 10 120 python3 -u tools/nf_ab.py --lib tools/ab_libs/libmmb_nf_$v.so --n 1284 --steps 50 >> $OUT/ab.txt 2>>$OUT/ab.err || exit 1
done; done
cat $OUT/ab.txt
