#!/bin/bash
# sweep_env.sh with a given libgsr.so: bash tools/sweep_env_lib.sh LIB VAR v1 v2 ...
set -u
lib=$1; shift
GSR_LIB=$lib bash tools/sweep_env.sh "$@"
