set -o pipefail
O=gpurun_out/r03z
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc $rc" >> $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python -u profiles/chain_tiles.py > $O/tiles.log 2>&1
