#!/bin/bash
# same-box A/B of two builds of the extension (gpubin/C_old.so, gpubin/C_new.so), alternating;
# each variant runs from its own copy of the package + scripts (so sys.path[0] is the copy)
# usage: [AB_VARIANTS="a b c"] gpubin/ab.sh <script> <args...>   (script path relative to the repo
# root; variant v runs gpubin/C_v.so; default "old new", each list run twice)
set -e
root=$PWD
script=$1; shift
vs=${AB_VARIANTS:-old new}
for v in $vs $vs; do
  d=/tmp/ab_$v
  rm -rf $d && mkdir -p $d && cp -r tensorflow_distributed_clustering_amd scripts bench.py $d/
  cp gpubin/C_$v.so $d/tensorflow_distributed_clustering_amd/_C.so
  echo "== $v"
  (cd $d && timeout -k 10 200 python $script "$@" 2>&1 | grep -v amdgpu.ids)
done
