#!/bin/bash
# Round 4: SURVEY 8(f) row 2 measured at scale -- device ingest + standardize and the device
# calc_A_hat build against the oracle's host restatements, bit-exact checks (tools/ingest_time.py).
set -u
tools/gpu_session.sh \
 "ingest_arxiv::300::python tools/ingest_time.py --workload arxiv-synth" \
 "ingest_products::600::python tools/ingest_time.py --workload products-synth"
