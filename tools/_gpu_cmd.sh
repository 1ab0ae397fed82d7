set -o pipefail
O=gpurun_out/pmc7; mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline"
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES --output-format csv -d $O/p1 -o run -- $B > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $O/p2 -o run -- $B > $O/p2.log 2>&1 || { tail -5 $O/p2.log; exit 1; }
timeout -k 10 200 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_BUSY_CYCLES --output-format csv -d $O/p3 -o run -- $B > $O/p3.log 2>&1 || { tail -5 $O/p3.log; exit 1; }
python tools/pmc_sq.py $O/p1 $O/p2 $O/p3
