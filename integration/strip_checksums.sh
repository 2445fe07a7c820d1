#!/bin/bash
# TEST INFRASTRUCTURE (integration/Makefile, target `dropin`): removes the
# reference's own checksum definitions from its compiled objects, so that a
# stack linked from them takes every checksum from libtulips_csum.so. No
# reference source is edited; only the objects built from it are.
#
#   usage: strip_checksums.sh <objdir>
#
# A definition no relocation in its object names is stripped; one its own
# object still calls (the tcpv4 verify site calls Processor::checksum in the
# same translation unit) is made weak instead, so the dynamic linker takes
# libtulips_csum.so's definition, which precedes the stack in lookup order.
set -euo pipefail
D=$1
pairs=(
  "stack/Utils.o _ZN6tulips5stack5utils8checksumEtPKht"
  "stack/IPv4.o _ZN6tulips5stack4ipv48checksumEPKh"
  "stack/ICMPv4.o _ZN6tulips5stack6icmpv48checksumEPKh"
  "stack/tcpv4/Processor.o _ZN6tulips5stack5tcpv49Processor8checksumERKNS0_4ipv47AddressES6_tPKh"
)
for p in "${pairs[@]}"; do
  set -- $p
  o=$D/$1; s=$2
  # compiled out by the gates (TULIPS_HAS_HW_CHECKSUM + DISABLE_CHECKSUM_CHECK)
  nm "$o" | grep -q " [TW] $s\$" || { echo "absent   $s ($1)"; continue; }
  if objcopy --strip-symbol="$s" "$o" 2>/dev/null && ! nm "$o" | grep -q " [TW] $s\$"; then
    echo "stripped $s ($1)"
  else
    objcopy --weaken-symbol="$s" "$o"
    echo "weakened $s ($1)"
  fi
done
