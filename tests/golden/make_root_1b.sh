#!/bin/bash
# Golden roots of BASELINE.json configs[3] (1B keys = 8 key-range shards of 125M records, 32-B keys /
# 100-B values, seed 0x4D65726B6C654B56, shard g = records [g*125M, (g+1)*125M) with key char 0 in the g-th
# eighth of the alphabet) and of its one-GPU share (125M = 8 x 15.625M), computed on the CPU by the oracle's
# streaming restatement (oracle/root_stream.c; ~3 min for 1B on 8 cores, 16 GB of RAM). Run in this
# container; the GPU tests only read the JSON.
set -e
cd "$(dirname "$0")/../.."
make -C oracle root_stream > /dev/null
{
  echo '{"generator": "oracle/root_stream SEED G NPER 32 100 20 8", "cases": ['
  oracle/root_stream 0x4D65726B6C654B56 8 125000000 32 100 20 8
  echo ','
  oracle/root_stream 0x4D65726B6C654B56 8 15625000 32 100 20 8
  echo ']}'
} > tests/golden/roots_sharded.json.tmp
python3 -c "import json; d=json.load(open('tests/golden/roots_sharded.json.tmp')); json.dump(d, open('tests/golden/roots_sharded.json','w'), indent=1)"
rm tests/golden/roots_sharded.json.tmp
