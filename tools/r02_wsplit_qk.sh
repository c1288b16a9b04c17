# Whisper attention weight-split refinement (q/k vs v vs out) on three seeds: de-normalised mel-L1 vs the fp32 oracle
set -o pipefail
mkdir -p gpurun_out
V="0x1fffffffffffff:15,0x1fffffffffffff:15:0xffffff:0:0xffffff,0x1fffffffffffff:15:0xffffff:0:0,0x1fffffffffffff:15:0xffffff:0xffffff:0"
for seed in 7 11; do
  timeout -k 10 500 python3 -u tools/precision_sweep.py --gpu --content whisper --no-emu --no-vocoder --seed $seed \
    --wsplit-variants "$V" > gpurun_out/wsqk_$seed.json 2> gpurun_out/wsqk_$seed.err || exit $?
  python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))
for k,v in d['results'].items(): print(sys.argv[2], round(v['mel_l1_denorm_ln']*1e3,4), k)" gpurun_out/wsqk_$seed.json $seed
done
