set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r06j
mkdir -p $O
timeout -s KILL 200 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum --kernel-trace -d $O/pmc -o run --output-format csv -- python3 -u tools/gpu/exact_line.py > $O/exact_pmc.json 2> $O/exact_pmc.err || { echo "pmc failed"; tail -5 $O/exact_pmc.err; exit 1; }
echo done
