set -u
# final device code: kernel statistics and the PMC passes of the two stateful headlines
bash tools/session.sh r06fin3 stats=config3 stats=config5 pmc=config3 pmc=config5 cal
