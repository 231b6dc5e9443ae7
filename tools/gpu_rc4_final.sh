set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/rc4final; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_rc4.py tests/test_batcher.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 && tail -1 $O/pytest.log &&
timeout -k 10 300 python3 bench.py --op rc4 > $O/rc4.json 2> $O/rc4.err && cat $O/rc4.json &&
timeout -k 10 300 python3 bench.py --op rc4md5 > $O/rc4md5.json 2> $O/rc4md5.err && cat $O/rc4md5.json
