set -o pipefail
bash scripts/sweep_chunks_steal.sh && bash scripts/occ_probe.sh
