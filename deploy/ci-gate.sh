#!/bin/bash
# CI gate (the reference's README.md:169-180 scenario): only submit the job when
# at least one MI355X node is Ready *and* healthy.
set -u
if check-gpu-node --mi355x --slack-only-on-error; then
    echo "GPU nodes ready; submitting"
    kubectl apply -f "${1:-ml-job.yaml}"
else
    rc=$?
    echo "no Ready+healthy MI355X node (exit $rc); not submitting" >&2
    exit 1
fi
