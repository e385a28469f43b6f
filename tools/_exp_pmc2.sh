set -u
cd "${GRAFT_REPO_ROOT:-.}"
G="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY"
bash tools/_exp_pmc.sh "$G" && cp gpurun_out/pmcx/summary.txt gpurun_out/pmc_new.txt && \
COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_pyrold.so bash tools/_exp_pmc.sh "$G" && cp gpurun_out/pmcx/summary.txt gpurun_out/pmc_old.txt
