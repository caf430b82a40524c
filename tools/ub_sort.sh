#!/bin/bash
for a in "9469536 23" "4000000 22" "1000000 19" "478000 18" "100000 16" "5000000 31" "2000 11" "3 2"; do
  tools/ubench_sort $a 20 || exit 1
done
