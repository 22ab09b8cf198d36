from .trainer import main

main()
