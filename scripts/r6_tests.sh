# round 6: the full -m gpu suite and smoke() on the tree as it is
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6t
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r6t/pytest.log 2>&1; rc=$?
tail -5 gpurun_out/r6t/pytest.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/r6t/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6t/smoke.log 2>&1; rc=$?
tail -3 gpurun_out/r6t/smoke.log
exit $rc
