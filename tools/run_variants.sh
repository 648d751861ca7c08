#!/bin/bash
# time tools/mlp_driver.py against each experiment library (tools/build_variants.py)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for v in ${VARIANTS:-base nodma noestore noeload noslab}; do
  echo -n "$v: "
  NR_LIB=neurecon_amd/_exp/libnrhip_$v.so timeout -k 10 120 python3 tools/mlp_driver.py ${DRIVER_ARGS} 2>&1 | tail -1 || exit 1
done
