set -eo pipefail
mkdir -p gpurun_out/g8
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 60 rocprofv3 --list-avail > gpurun_out/g8/avail.txt 2>&1 || true
grep -c . gpurun_out/g8/avail.txt
