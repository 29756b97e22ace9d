# Chebyshev launch A/B under rocprofv3 (kernel trace + WRITE_SIZE per variant): VARS="k=v;k=v ..."
set -o pipefail
O=gpurun_out/cheb_pmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
i=0
IFS=';' read -ra VS <<< "${VARS:-EIGMI_NOTHING=1}"
for v in "${VS[@]}"; do
  i=$((i+1))
  env_args=$(echo "$v" | tr ',' ' ')
  export $env_args
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/t$i -o tr -- python3 tools/cheb_sweep.py --rounds 1 > $O/v$i.json 2> $O/v$i.err || exit 1
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w$i -o pmc -- python3 tools/cheb_sweep.py --rounds 1 > /dev/null 2>> $O/v$i.err || exit 1
  unset $(echo "$env_args" | sed 's/=[^ ]*//g')
  echo "$i $v" >> $O/variants.txt
done
