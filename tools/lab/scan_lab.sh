#!/bin/bash
# tools/lab/scan_lab.sh — whole-file scrub (page_checksum_tool --scan) rate on
# a 1 GiB and a 4 GiB file of 4 KiB pages (page cache warm) against reader
# threads / read piece / chunk size.  Not part of the product.
set -euo pipefail
TOOL=eloqstore_amd/page_checksum_tool
D=$(mktemp -d /tmp/scanlab.XXXX)
trap 'rm -rf "$D"' EXIT
timeout -k 10 120 $TOOL --gen "$D/f1" 262144 4096 0x5EED0001 > /dev/null
timeout -k 10 120 $TOOL --gen "$D/f4" 1048576 4096 0x5EED0001 > /dev/null
cat "$D/f1" "$D/f4" > /dev/null  # warm the page cache
for f in f1 f4; do
  for cfg in "8 8 64" "16 8 64" "16 4 64" "16 8 128"; do
    set -- $cfg
    for rep in 1 2 3; do
      line=$(PCS_SCAN_THREADS=$1 PCS_SCAN_PIECE_MIB=$2 PCS_SCAN_CHUNK_MIB=$3 timeout -k 10 120 $TOOL --scan "$D/$f")
      echo "$f threads=$1 piece=$2MiB chunk=$3MiB rep=$rep: $line"
    done
  done
done
