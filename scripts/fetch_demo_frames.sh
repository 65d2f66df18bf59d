#!/bin/bash
# The repo ships demo-Game (10 frames), demo-static (15) and the first 20 frames of demo-Cat /
# demo-YogaHut2 (the reference's demo inputs, `SURVEY.md` §2.1 #55).  Copy the complete sequences
# (100 / 250 frames) from a checkout of the reference:  scripts/fetch_demo_frames.sh <ref_dir>
set -e
REF=${1:?usage: fetch_demo_frames.sh <reference checkout>}
cd "$(dirname "$0")/.."
for d in demo-Game demo-static demo-Cat demo-YogaHut2; do
  mkdir -p "$d"
  cp -n "$REF/$d"/* "$d"/
  echo "$d: $(ls "$d" | wc -l) frames"
done
