set -u
# the final build's headline spread: config 3 twice more, config 5 once more (fresh box)
bash tools/session.sh r06p bench=config3 bench=config3,--steps,20 bench=config5
