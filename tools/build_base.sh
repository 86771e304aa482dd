#!/usr/bin/env bash
# Build the diagnostic library of a committed revision (default HEAD) as
# keypoint-detection_amd/dll/_lib/libkpd_base.so, for same-box A/B of an
# uncommitted kernel change against it:
#   tools/build_base.sh [rev]
#   AB_ENVS="-;KPD_LIB=keypoint-detection_amd/dll/_lib/libkpd_base.so" STEPS=ab bash tools/gpu_session.sh
set -eu
ROOTD="$(cd "$(dirname "$0")/.." && pwd)"
REV="${1:-HEAD}"
T=$(mktemp -d /tmp/kpd_base.XXXX)
git -C "$ROOTD" archive "$REV" keypoint-detection_amd/csrc include | tar -x -C "$T"
make -C "$T/keypoint-detection_amd/csrc" -j8 diag OUT_DIAG="$ROOTD/keypoint-detection_amd/dll/_lib/libkpd_base.so" >/dev/null
rm -rf "$T"
echo "built libkpd_base.so from $REV"
