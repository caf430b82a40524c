cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp KLSH_MERGE_STREAMS=0
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU --output-format csv --kernel-include-regex "k_merge_small|k_project_pk" -d gpurun_out/pmcs1 -o run -- python bench.py --steps 1 --warmup 0 --iterations 60 --cpu-baseline none > gpurun_out/pmcs1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE --output-format csv --kernel-include-regex "k_merge_small|k_project_pk" -d gpurun_out/pmcs2 -o run -- python bench.py --steps 1 --warmup 0 --iterations 60 --cpu-baseline none > gpurun_out/pmcs2.log 2>&1 || exit 1
echo done
