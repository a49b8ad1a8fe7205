#!/bin/bash
# Build-container side of tools/profile_r6_pmc.sh: one profiles/r6p_<case>_summary.json (+ kernel
# stats CSV) per case and its entry in profiles/pmc_traffic.json, keyed by the traffic_key its
# bench line printed.
set -eu
cd "$(dirname "$0")/.."
for d in gpurun_out/pmc/*/; do
  tag=$(basename "$d")
  [ -f "gpurun_out/${tag}_stats.log" ] || continue
  wl=products-synth
  case $tag in pubmed) wl=pubmed-synth ;; msacad) wl=ms-academic-synth ;; esac
  python tools/summarize_profile.py "r6p_$tag" "$d/stats" "$d/fetch" "$d/write" \
    --workload "$wl" --bench-json "gpurun_out/${tag}_stats.log" > /dev/null
  echo "r6p_$tag"
done
