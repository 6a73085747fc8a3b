# round 6: DPM clock levels (read-only sysfs) through the backend-gap phases
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6dpm
for d in /sys/bus/pci/devices/*/pp_dpm_mclk; do echo "$d"; done | head -3 > gpurun_out/r6dpm/sysfs.txt
for ph in res_b2b res_gap2 res_fresh res_fresh_sleep10 res_fresh_other; do
  MOSRX_DPM_WATCH=1 timeout -k 10 120 python3 -u scripts/diag_backend_gap.py M1500c8 $ph >> gpurun_out/r6dpm/dpm.log 2>&1 || { tail -20 gpurun_out/r6dpm/dpm.log; exit 1; }
done
cat gpurun_out/r6dpm/sysfs.txt
grep -v "^\[" gpurun_out/r6dpm/dpm.log | cut -c1-1500
