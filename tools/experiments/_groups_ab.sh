for r in 1 2; do for g in 1 2 3 4; do
  out=$(ICP4R_GROUPS=$g timeout -k 10 120 python3 bench.py --no-cpu --no-upload --no-c5 --check 2 --steps 20 2>/dev/null | grep '^{')
  python3 -c "import json,sys; r=json.loads(sys.argv[1]); print('groups', sys.argv[2], round(r['value']), r['parity_ok'])" "$out" $g
done; done
