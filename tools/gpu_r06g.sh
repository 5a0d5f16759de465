set -u
bash tools/session.sh r06g ab=config5,main,cont3,w3,npos3,cont2,main,cont3
