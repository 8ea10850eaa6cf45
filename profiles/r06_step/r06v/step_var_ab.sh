set -e
O=gpurun_out/r06v; mkdir -p $O
for i in 1 2 3; do
  for lib in base new vfk van vboth; do
    L=libexo_amd_$lib.so; [ $lib = new ] && L=libexo_amd.so
    EXO_AMD_LIB=$L timeout -k 10 180 python3 -u tools/step_ab.py $O/${lib}_rows_$i --rounds 10 > $O/${lib}_rows_$i.log 2>&1
    EXO_AMD_LIB=$L timeout -k 10 180 python3 -u tools/step_ab.py $O/${lib}_shared_$i --rounds 10 --variant rows_shared > $O/${lib}_shared_$i.log 2>&1
  done
done
