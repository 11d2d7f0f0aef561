#!/bin/bash
# Compare the gfx950 ISA of every kernel between a saved snapshot and the current build (the
# instruction text per function: addresses, encodings and branch-target labels stripped).  A code
# change meant to leave the kernels' instruction streams alone must print "identical" for them.
# (s_add_u32 / s_addc_u32 literals are PC-relative offsets after s_getpc_b64 -- they move with the
# size of other kernels in the code object -- and are masked.)
# usage: scripts/isa_compare.sh save DIR | compare DIR
set -eu
B=${ISA_BUILD:-mini-opencl-raytracer_amd/build}  # (ISA_BUILD: a variant's object directory)
LLVM=/opt/rocm/lib/llvm/bin
dump() {  # dump OUTDIR
  mkdir -p $1
  for o in rt_kernels_shipped rt_kernels; do
    cp $B/$o.o $1/
    (cd $1 && $LLVM/llvm-objdump --offloading $o.o > /dev/null && mv $o.o.0.hipv4-amdgcn-amd-amdhsa--gfx950 $o.co && rm -f $o.o.0.host* $o.o)
    $LLVM/llvm-objdump -d --no-show-raw-insn $1/$o.co \
      | sed -E 's#[[:space:]]*//.*$##; s/<[^>]*\+0x[0-9a-f]+>//g; s/^(.*s_addc?_u32 .*, )0x[0-9a-f]+$/\1REL/' \
      | awk '/^[0-9a-f]+ <.*>:$/ {name=$2; next} name != "" {$1 = $1; if (NF) print name "\t" $0}' > $1/$o.isa
  done
}
case $1 in
  save) rm -rf $2; dump $2 ;;
  compare)
    rm -rf /tmp/isa_now
    dump /tmp/isa_now
    for o in rt_kernels_shipped rt_kernels; do
      for f in $(cut -f1 $2/$o.isa | sort -u); do
        a=$(grep -F "$f" $2/$o.isa | cut -f2- | md5sum | cut -c1-12)
        b=$(grep -F "$f" /tmp/isa_now/$o.isa | cut -f2- | md5sum | cut -c1-12)
        n=$(grep -cF "$f" /tmp/isa_now/$o.isa || true)
        [ "$a" = "$b" ] && echo "identical  $o $f" || echo "CHANGED    $o $f ($n insts now)"
      done
    done ;;
esac
