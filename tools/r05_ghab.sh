#!/bin/bash
# defaults vs gram_huge_min=256 and vs the round-4 lead substitution grid (sub_grid_lead=80, the
# old fixed 5/16 of the CUs), configs 4 / 5 / 3, two alternating rounds on one box
set -u
for r in 1 2; do
  for c in 4 5 3; do
    echo "round $r config $c"
    bash tools/ab_opts.sh $c "" "gram_huge_min=256" "sub_grid_lead=80" || exit 1
  done
done
echo done
