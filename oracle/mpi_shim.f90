module mpi
    include 'mpif.h'
end module mpi
