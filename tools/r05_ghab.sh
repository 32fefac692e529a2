#!/bin/bash
# gram_huge_min default (384) vs 256 / 192, configs 4 / 5 / 3, three alternating rounds on one box
set -u
for r in 1 2 3; do
  for c in 4 5 3; do
    echo "round $r config $c"
    bash tools/ab_opts.sh $c "" "gram_huge_min=256" "gram_huge_min=192" || exit 1
  done
done
echo done
