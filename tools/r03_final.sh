#!/bin/bash
# Round-3 validation on one box: GPU tests, smoke, default bench, then the
# kernel trace + PMC passes of the bench (tools/profile.sh).  Stops at the first failure.
set -u
TAG=${1:-r03}
R=$GRAFT_REPO_ROOT
cd $R
bash tools/validate.sh $TAG || exit $?
bash tools/profile.sh $TAG --steps 5 --warmup 2 --no-cpu --no-secondary || exit 10
echo all done
