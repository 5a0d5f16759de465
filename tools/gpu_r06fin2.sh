set -u
# final device code: the bench lines (headline first)
bash tools/session.sh r06fin2 bench=config3 bench=config5 bench=config1 bench=config2 \
  bench=config3,--ct-max-log2,26,--gc-step,61 bench=config3,--zipf,1.1 bench=config3,--ct-room,0 \
  bench=config5,--ct-local,64000 bench=config5,--ct-local,64000,--ep-zipf,0.6 \
  bench=config3,--ct-local,64000,--ep-zipf,1.0 bench=config5,--ct-max,1000000 bench=config5,--ep-owned
