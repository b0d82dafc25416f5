#!/bin/bash
# tools/ab.sh on one rank's share of the C2 frame under the strong-scaling
# tile deal.  usage: tools/ab_share.sh <world> <rounds> lib1.so lib2.so ...
world=$1; shift
QB_ARGS="--tiles --spp 1000 --world $world --rank 0" exec bash "$(dirname "$0")/ab.sh" "$@"
