#!/bin/bash
# Build timing variants of libgnnrec.so: variants.sh NAME "EXTRA hipcc flags" ...
# -> tools/_diag/libgnnrec_NAME.so (same soname, load with GNNREC_LIB=...)
set -e
cd "$(dirname "$0")/../../gnn-recsys_amd/csrc"
while [ $# -ge 2 ]; do
  make -s -j8 OBJDIR=build_$1 OUT=../../tools/_diag/libgnnrec_$1.so EXTRA="$2" ../../tools/_diag/libgnnrec_$1.so
  shift 2
done
