# round-5 A/B session 3: the world-1 gather flow (copy-ipc) with 2 (main), 4 and 8 transfer streams
set -u
DIST_TAG=xfer bash scripts/dist_ab.sh 3 --transport copy-ipc || exit 1
