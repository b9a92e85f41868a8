for v in base NO_REDUCE NO_DOT NO_STORE NO_LL NO_POSTNORM NO_LL_NO_POSTNORM; do
  if [ $v = base ]; then L=nip_amd/_lib/libnip_amd.so; else L=nip_amd/_lib/abl_$v.so; fi
  NIPAMD_LIB=$L timeout -k 10 120 python bench.py --no-cpu-baseline --no-check 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['roofline']['kernel_ms'],4), '%.3g'%d['value'])"
done
