# A/B: kernel arguments in device memory (the HIP runtime's default here) or in host memory
# (HIP_FORCE_DEV_KERNARG=0), on the small-batch legs (launch-bound: tools/host_gaps.py) and cfg5.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r5ka}; mkdir -p $out
for r in 1 2; do
  for v in dflt 0; do
    for leg in cfg2 cfg3; do
      if [ $v = dflt ]; then
        timeout -k 10 120 python bench.py --only $leg --steps 200 > $out/${leg}_${v}_$r.json 2>$out/err.log || exit 1
      else
        HIP_FORCE_DEV_KERNARG=$v timeout -k 10 120 python bench.py --only $leg --steps 200 > $out/${leg}_${v}_$r.json 2>$out/err.log || exit 1
      fi
      echo "$leg $v $r $(python -c "import json,sys; print(json.load(open('$out/${leg}_${v}_$r.json'))['value'])")"
    done
  done
done
for v in dflt 0; do
  if [ $v = dflt ]; then
    timeout -k 10 300 python bench.py --no-cpu --no-e2e --no-live --no-legs --no-decode --steps 20 > $out/cfg5_$v.json 2>$out/err.log || exit 1
  else
    HIP_FORCE_DEV_KERNARG=$v timeout -k 10 300 python bench.py --no-cpu --no-e2e --no-live --no-legs --no-decode --steps 20 > $out/cfg5_$v.json 2>$out/err.log || exit 1
  fi
  echo "cfg5 $v $(python -c "import json; print(json.load(open('$out/cfg5_$v.json'))['value'])")"
done
