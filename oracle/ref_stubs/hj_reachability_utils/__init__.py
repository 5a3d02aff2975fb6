"""hj_reachability_utils stub (never vendored by the reference, README.md:38-40)."""
