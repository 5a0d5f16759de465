set -u
CV_ADMIT_STATS=1 bash tools/session.sh r06j stats=config5,--ct-local,64000,--ep-zipf,0.6
