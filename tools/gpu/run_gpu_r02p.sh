#!/bin/bash
# drain write pass variants: LDS image 48/32/24 KB (3/4/5 workgroups per CU) x plain / non-temporal stores
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r02p
cp zeebe_amd/libzbgpu.so gpurun_out/r02p/keep.so
for v in img48_w3 img32_w4 img24_w5; do
  cp variants/libzbgpu_$v.so zeebe_amd/libzbgpu.so
  for nt in 0 1; do
    ZB_SER_NT=$nt timeout -k 10 300 python3 -u bench.py --no-extras --no-cpu-baseline --steps 4 > gpurun_out/r02p/$v.nt$nt.json 2> gpurun_out/r02p/$v.nt$nt.err || { echo "$v nt=$nt failed"; tail -5 gpurun_out/r02p/$v.nt$nt.err; cp gpurun_out/r02p/keep.so zeebe_amd/libzbgpu.so; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/r02p/$v.nt$nt.json'));b=d['step_breakdown_ms'];print('$v nt=$nt', round(d['value']/1e9,3), round(d['ms_per_step'],3), round(b['drain_write_kernel'],3), round(b['drain_size_kernel'],3))"
  done
done
cp gpurun_out/r02p/keep.so zeebe_amd/libzbgpu.so
