set -u
cd /root/repo
for r in 1 2; do
  for d in . _ab; do
    out=$(cd $d && timeout -k 10 300 python bench.py --config c3 --steps 30 --warmup 5 --no-cpu-baseline --no-c5 --no-caption-mode --no-eot-mode 2>/dev/null)
    rc=$?; [ $rc -eq 0 ] || { echo "$d rc=$rc"; exit $rc; }
    echo "$d $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["fedavg_round_wall"]["c3"]; print(round(d["value"],1), "img/s", round(d["ms_per_step"],3), "ms; round", round(r["round_wall_s"],3), "s train", round(r["split_s"]["local_train_s"],3), "test", round(r["split_s"]["local_test_s"],3))')"
  done
done
