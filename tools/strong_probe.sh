for spec in "1250 -1" "1250 10" "1250 11" "1250 12" "1250 6" "2500 -1" "10000 -1"; do
  set -- $spec
  r=$(timeout -k 10 120 python bench.py --no-cpu-baseline --no-pgo --steps 10 --pairs $1 --instance $2 2>/dev/null) || { echo "$spec FAILED"; exit 1; }
  echo "pairs $1 inst $2 $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"])')"
done
