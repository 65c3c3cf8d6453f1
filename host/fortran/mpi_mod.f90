! The `mpi` module for flang: MPICH's public mpif.h (MPICH ships a gfortran-format mpi.mod).
module mpi
    include 'mpif.h'
end module mpi
