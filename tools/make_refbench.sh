#!/bin/bash
# Pack the unmodified reference source (read-only checkout) into .refbench/ref_src.tar.gz for the reference-timing
# tools (tools/ref_bench.py, tools/domain_bench.py, tools/ref_config_bench.py).  The tarball is git-ignored: the
# reference's code is only ever run for timing / parity, never copied into this package.
set -eu
REF=${1:-/root/reference}
cd "$(dirname "$0")/.."
mkdir -p .refbench
tar -czf .refbench/ref_src.tar.gz -C "$REF" src/torchmetrics
echo "wrote .refbench/ref_src.tar.gz"
