#!/bin/bash
# drain write pass: flat (generic-pointer) encoder vs LDS-typed encoder (ds_write), NT stores on
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r02q
cp zeebe_amd/libzbgpu.so gpurun_out/r02q/keep.so
for v in img48_w3 lds; do
  cp variants/libzbgpu_$v.so zeebe_amd/libzbgpu.so
  ZB_SER_NT=1 timeout -k 10 300 python3 -u bench.py --no-extras --no-cpu-baseline --steps 4 > gpurun_out/r02q/$v.json 2> gpurun_out/r02q/$v.err || { echo "$v failed"; tail -5 gpurun_out/r02q/$v.err; cp gpurun_out/r02q/keep.so zeebe_amd/libzbgpu.so; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r02q/$v.json'));b=d['step_breakdown_ms'];print('$v', round(d['value']/1e9,3), round(d['ms_per_step'],3), round(b['drain_write_kernel'],3), round(b['drain_size_kernel'],3))"
done
cp gpurun_out/r02q/keep.so zeebe_amd/libzbgpu.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_frames.py tests/test_gpu_iomapping.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r02q/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r02q/tests.log; exit 1; }
tail -1 gpurun_out/r02q/tests.log
