#!/bin/bash
# C3-geometry A/B (2048^2, 16 spp, 1000 spheres) of librtp builds: tools/ab.sh with C3 arguments.
QB_ARGS="--nx 2048 --ny 2048 --spp 16 --variant 3" exec tools/ab.sh "$@"
