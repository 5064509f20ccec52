set -u
for L in ${LIBS:-base nofrag allno}; do
  if [ $L = base ]; then lib=tensorium_amd/libtensorium_hip.so; else lib=ab/$L/libtensorium_hip.so; fi; A=${NB_ARGS:-}
  echo "== $L"; TNS_LIB=$lib timeout -k 10 100 python scripts/nn_big_ab.py --variants 0 --rounds 3 $A 2>&1 | grep -A2 '"256x256x32_w2x4' | grep ms_median || exit 1
done
