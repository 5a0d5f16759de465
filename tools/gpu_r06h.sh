set -u
bash tools/session.sh r06h ab=config5,main,lb5,lb3,pairs5,main
