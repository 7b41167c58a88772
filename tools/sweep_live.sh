# k_liveness chunks-per-workgroup sweep (LIVE_PER build variants under aiocluster_amd/lib/var/)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sweep_live
for v in default 4 16 32 default; do
  if [ $v = default ]; then lib=""; else lib=aiocluster_amd/lib/var/lp$v.so; fi
  GS_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/sweep_live/lp_$v.$RANDOM.log 2>&1 || exit 1
done
