#!/bin/bash
# usage: scripts/isa_stats.sh <file.hip> <kernel-name-regex>  -> instruction counts of one kernel
set -e
f=$(readlink -f "$1"); pat=$2
d=$(mktemp -d); cd "$d"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -x hip -c "$f" -o k.o -save-temps >/dev/null 2>&1
S=$(ls *gfx950.s)
name=$(grep -oE "^_ZN[^:]*${pat}[^:]*:" "$S" | head -1 | tr -d :)
awk -v n="$name:" '$1==n,/s_endpgm/' "$S" > k.s
echo "$name: $(wc -l < k.s) lines"
for p in v_fma_f64 v_mfma s_load global_load buffer_load ds_read ds_write ds_bpermute s_waitcnt s_barrier scratch; do printf "%-14s %s\n" $p $(grep -c "$p" k.s || true); done
grep -E "vgpr_count|sgpr_count|spill" "$S" | grep -A0 "" | head -0
cp k.s /tmp/last_kernel.s
