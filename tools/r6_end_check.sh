#!/bin/bash
# Round 6 end: the round-end check (GPU tests, smoke, bench line, WBC bench line, N = 2 rehearsal) and a longer
# randomised parity sweep (tools/fuzz_parity.py, batch 1024).  Output under gpurun_out/rc/ and gpurun_out/end/.
bash tools/round_check.sh || exit $?
mkdir -p gpurun_out/end
timeout -k 10 330 python tools/fuzz_parity.py --seconds 240 --batch 1024 --out gpurun_out/end/fuzz_b1024.json > gpurun_out/end/fuzz_b1024.log 2>&1 || exit 8
python -c "import json; d=json.load(open('gpurun_out/end/fuzz_b1024.json')); print({k: d[k] for k in d if not isinstance(d[k], (list, dict))})"
