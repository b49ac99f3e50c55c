#!/bin/bash
# Per-kernel wait census of the BSR kernels' ISA: for each mangled-name
# fragment given, the s_waitcnt lines after the kernel's 2nd s_barrier (the
# steady-state loop onward), plus VGPR / AGPR / LDS usage.
# usage: tools/isa_waits.sh <name-fragment>...   (after `make asm`-style build)
S=${S:-$(dirname "$0")/../spmm-denseblock_amd/build/asm/bsr_kernels-hip-amdgcn-amd-amdhsa-gfx950.s}
for K in "$@"; do
  echo "== $K"
  awk -v k="$K" '$0 ~ "^_Z.*"k && $0 ~ /:/ && !f {f=1} /^\.Lfunc_end/{if(f)exit} f' "$S" |
    awk '/s_barrier/{c++} c>=2' | grep -E "s_waitcnt" | sort | uniq -c
  grep -E "^\s+\.set .*$K.*\.(num_vgpr|num_agpr)," "$S" | head -2 | awk '{print "  ", $2, $3}'
  grep -A40 "\.amdhsa_kernel .*$K" "$S" | grep -m1 group_segment_fixed_size
done
