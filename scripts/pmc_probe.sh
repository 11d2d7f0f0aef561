# rocprofv3: available counters (to a file) and the default profile (scripts/profile.sh) of the
# headline and the bunny proxy
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 --list-avail > gpurun_out/rocprof_avail.txt 2>&1 || true
bash scripts/profile.sh cornell_r03 || exit 1
bash scripts/profile.sh bunny_r03 --scene bunny || exit 1
