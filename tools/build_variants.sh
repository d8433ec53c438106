# Build libphantom_amd variants with NTT tuning knobs into tools/variants/<name>/lib (experiments only)
set -e
ROOT=$(cd $(dirname $0)/.. && pwd)
build() {
  name=$1; shift
  d=$ROOT/tools/variants/$name
  rm -rf $d && mkdir -p $d && cp -r $ROOT/phantom-fhe-boot_amd/csrc $ROOT/phantom-fhe-boot_amd/host $ROOT/phantom-fhe-boot_amd/examples $ROOT/phantom-fhe-boot_amd/Makefile $d/
  mkdir -p $d/py && cp $ROOT/phantom-fhe-boot_amd/py/phantom_amd.py $d/py/
  make -C $d -j4 INCDIR=$ROOT/include EXTRA="$*" lib/libphantom_amd.so > $d/build.log 2>&1
  echo built $name
}
rm -rf $ROOT/tools/variants
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  build $name $flags &
done
wait
