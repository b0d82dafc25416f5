#!/bin/bash
# tools/ab.sh on bench.py's instance (C2, tile deal, jump tables on).
# usage: tools/ab_c2_tiles.sh <rounds> lib1.so lib2.so ...   ("main" = in-tree librtp.so)
QB_ARGS="--tiles --spp 1000" exec bash "$(dirname "$0")/ab.sh" "$@"
