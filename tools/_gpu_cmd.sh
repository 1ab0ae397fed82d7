set -o pipefail
O=gpurun_out/pro1; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python tools/ab_variants.py --rounds 7 base= pro_all=-DG2K_DIAG_PROLOGUE=1 pro_weights=-DG2K_DIAG_PROLOGUE=2 pro_pos=-DG2K_DIAG_PROLOGUE=3 > $O/ab.log 2>&1 || { tail -30 $O/ab.log; exit 1; }
grep median $O/ab.log
