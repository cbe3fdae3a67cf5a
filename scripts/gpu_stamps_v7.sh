cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
MLG_ROLLOUT_KERNEL=v7 MLG_LIB=ma-league_amd/maleague/_lib/libmaleague_stamps.so timeout -k 10 300 python scripts/stamps_rollout.py > gpurun_out/stamps_v7.txt 2>&1 || { echo "stamps failed"; tail -20 gpurun_out/stamps_v7.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/stamps_v7.txt | head -60
MODE=ai bash scripts/gpu_traffic.sh
