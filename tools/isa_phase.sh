#!/bin/bash
# Static instruction mix per phase of k_env_step<2,100> (between the STAMP s_memtime markers).
cd "$(dirname "$0")/../jaxmarl-hft_amd/csrc"
hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -DHFTLOB_STAMPS -S -o /tmp/hs.s hftlob.hip --cuda-device-only 2>/dev/null
L=$(grep -n "^_Z10k_env_stepILi2ELi100.*:" /tmp/hs.s | cut -d: -f1)
awk -v s=$L 'NR>=s' /tmp/hs.s | awk '/s_endpgm/{print; exit} {print}' > /tmp/ess.s
grep -n s_memtime /tmp/ess.s | cut -d: -f1 | tr '\n' ' ' > /tmp/stamps.txt
read -a M < /tmp/stamps.txt
names=(setup book rewards store)
for i in 0 1 2 3; do
  sed -n "${M[$i]},${M[$((i+1))]}p" /tmp/ess.s > /tmp/phase_$i.s
  f=/tmp/phase_$i.s
  echo "${names[$i]}: lines $(wc -l < $f) v_ $(grep -cE '^\s+v_' $f) s_ $(grep -cE '^\s+s_(add|sub|and|or|xor|andn2|orn2|not|mov|cselect|cmp|ff1|lshl|lshr|ashr|mul|min|max|bfe|bitcmp|cmov|abs)' $f) ds_ $(grep -cE '^\s+ds_' $f) br $(grep -cE '^\s+s_(cbranch|branch)' $f)"
done
