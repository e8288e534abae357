#!/bin/bash
# Round-end profiles of every bench config at the final library (run under
# gpurun): rocprofv3 kernel stats + the FETCH_SIZE / WRITE_SIZE passes per
# config (tools/profile_round.sh); summarise with tools/pmc_summary.py.
#   usage: final_prof.sh ROUND CONFIG...   (CONFIG: c3 | d2 | c2 | c4 | c5)
set -o pipefail
R=$GRAFT_REPO_ROOT
RN=$1; shift
for cfg in "$@"; do
  case $cfg in
    c3) args="" ; tag=$RN ;;
    d2) args="--data d2" ; tag=${RN}_d2 ;;
    *)  args="--config $cfg" ; tag=${RN}_$cfg ;;
  esac
  bash $R/tools/profile_round.sh $tag $args || { echo "profile $cfg failed"; exit 1; }
done
echo done
