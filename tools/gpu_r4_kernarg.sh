# round 4: where the kernel arguments live -- bench step with HIP_FORCE_DEV_KERNARG unset / 1 / 0
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for v in unset 1 0; do
    if [ $v = unset ]; then
      timeout -k 10 300 python -u bench.py --cpu-baseline 0 --no-prof --steps 20 > gpurun_out/r4_ka_$v$r.log 2> gpurun_out/r4_ka_$v$r.err || { tail -5 gpurun_out/r4_ka_$v$r.err; exit 1; }
    else
      HIP_FORCE_DEV_KERNARG=$v timeout -k 10 300 python -u bench.py --cpu-baseline 0 --no-prof --steps 20 > gpurun_out/r4_ka_$v$r.log 2> gpurun_out/r4_ka_$v$r.err || { tail -5 gpurun_out/r4_ka_$v$r.err; exit 1; }
    fi
    python -c "import json;d=json.load(open('gpurun_out/r4_ka_$v$r.log'));print('HIP_FORCE_DEV_KERNARG=$v', d['value'], d['ms_per_step'])"
  done
done
hipcc --offload-arch=gfx950 -O3 tools/kernarg_probe.hip -o /tmp/kernarg_probe > /dev/null 2>&1 || exit 1
timeout -k 10 120 /tmp/kernarg_probe > gpurun_out/r4_kernarg_probe.log 2>&1 || { tail -5 gpurun_out/r4_kernarg_probe.log; exit 1; }
cat gpurun_out/r4_kernarg_probe.log
HIP_FORCE_DEV_KERNARG=0 timeout -k 10 120 /tmp/kernarg_probe > gpurun_out/r4_kernarg_probe_host.log 2>&1 || { tail -5 gpurun_out/r4_kernarg_probe_host.log; exit 1; }
echo "HIP_FORCE_DEV_KERNARG=0:"; cat gpurun_out/r4_kernarg_probe_host.log
