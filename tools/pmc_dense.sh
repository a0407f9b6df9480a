#!/bin/bash
# PMC evidence for the dense MPNN kernels: SQ counters of one training forward
# (save), one inference forward and one backward at the bench's M=2048 ER-200 shape
# (tools/phase_timing.py with the product library), one rocprofv3 pass per counter group.
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
export ECO_HIP_LIB=$ROOT/eco-dqn_amd/eco_hip/libecohip.so
bash "$ROOT/tools/pmc_probe.sh" dense \
  "SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES" \
  "SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
  > "$ROOT/gpurun_out/pmc_dense.txt" 2>&1
rc=$?
cat "$ROOT/gpurun_out/pmc_dense.txt"
exit $rc
