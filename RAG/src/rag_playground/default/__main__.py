from generativeaiexamples_amd.playground.__main__ import main

if __name__ == "__main__":
    main()
