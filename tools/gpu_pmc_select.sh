set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcs
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d gpurun_out/pmcs/a -o a -- python3 tools/k1_batch1.py detect > gpurun_out/pmcs/a.log 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmcs/b -o b -- python3 tools/k1_batch1.py detect > gpurun_out/pmcs/b.log 2>&1
echo ok
