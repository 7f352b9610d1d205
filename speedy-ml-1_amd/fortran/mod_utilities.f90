!> mod_utilities -- the reference's shared derived types and grid constants
!> (src/mod_utilities.f90:1-631) for hosts that link the GPU path instead of the
!> reference's CPU reservoir code.  Same module name, type names, component names,
!> kinds and default initialisations, so the reference's callers of
!> speedy_res_interface (parallelmain.f90:9 `res%model_parameters`, `res%grid(i,j)`;
!> mod_reservoir.f90:334,614 and mod_slab_ocean_reservoir.f90:275 `reservoir`,
!> `grid`, `model_parameters`, `era_data`) type-check against this module unchanged.
!>
!> What is deliberately not here:
!>   * reservoir_type's MKL handles `cooA` (SPARSE_MATRIX_T) and `descrA`
!>     (MATRIX_DESCR), :185-186: the sparse A lives on the GPU (sml_res_create /
!>     sml_res_load_region_*, ELL + CSR), so no MKL module is needed to compile a
!>     caller;
!>   * the module's procedures (standardize_data*, gaussian_noise, init_random_seed,
!>     ...): the CPU data-preparation code of training and of the reference's host
!>     loop; the hot path's standardisation runs in the tiling kernels
!>     (sml_res_tile_*), its unstandardisation in the readout epilogue.
module mod_utilities
  use iso_fortran_env, only: int32
  implicit none

  integer, parameter :: dp = selected_real_kind(14)        ! :9
  integer, parameter :: sp = selected_real_kind(6, 37)     ! :10
  integer, parameter :: int_32 = int32                      ! :11
  real(kind=dp), parameter :: e_constant = 2.7182818284590452353602874_dp

  ! the T30 grid every rank shares (:17-20)
  integer :: speedygridnum = 96 * 48
  integer(kind=int32) :: xgrid = 96, ygrid = 48, zgrid = 8

  !> one reservoir's slice of the global grid (:32-164): resolved extents (res_*),
  !> their position in the local input tile (tdata_*), the overlap input extents
  !> (input_*), and the feedback vector's index ranges per variable
  type grid_type
    integer :: res_xstart, res_xend, res_ystart, res_yend, res_zstart, res_zend
    integer :: resxchunk, resychunk, reszchunk
    integer :: tdata_xstart, tdata_xend, tdata_ystart, tdata_yend, tdata_zstart, tdata_zend
    integer :: input_xstart, input_xend, input_ystart, input_yend, input_zstart, input_zend
    integer :: inputxchunk, inputychunk, inputzchunk
    logical :: pole, periodicboundary, top_vert_level, bottom_vert_level
    integer :: overlap, num_vert_levels, vert_overlap
    character(len=:), allocatable :: region_char
    real(kind=dp), allocatable :: mean(:), std(:)
    integer :: tisr_mean_std_idx, logp_mean_std_idx, sst_mean_std_idx, precip_mean_std_idx
    integer :: number_of_regions
    logical :: top, bottom
    integer :: level_index
    logical :: logp_bool
    integer :: atmo3d_start, atmo3d_end, sst_start, sst_end, logp_start, logp_end
    integer :: precip_start, precip_end, tisr_start, tisr_end, predict_start, predict_end
    integer :: othc_start, othc_end
  end type grid_type

  !> one reservoir (:166-367): hyper-parameters, COO A, W_in / W_out, states,
  !> training accumulators, input-composition flags and sizes, and the prediction
  !> loop's vectors (feedback, local_model, outvec, v_ml, v_p)
  type reservoir_type
    integer :: assigned_region
    integer, allocatable :: vert_indices_res(:), vert_indices_input(:)
    real(kind=dp), allocatable :: trainingdata(:, :)
    real(kind=dp) :: deg, radius, beta_res, beta_model, density, sigma, leakage
    integer, allocatable :: rows(:), cols(:)
    real(kind=dp), allocatable :: vals(:)
    integer :: k, reservoir_numinputs, locality, m, n
    real(kind=dp), allocatable :: win(:, :), wout(:, :), states(:, :), augmented_states(:, :)
    integer :: batch_size
    real(kind=dp), allocatable :: states_x_states(:, :), states_x_trainingdata(:, :)
    real(kind=dp), allocatable :: states_x_states_aug(:, :), states_x_trainingdata_aug(:, :)
    integer :: local_heightlevels_res, local_heightlevels_input, local_predictvars
    integer :: logp_size_res, logp_size_input
    logical :: logp_bool
    real(kind=dp), allocatable :: saved_state(:), current_state(:)
    logical :: tisr_input_bool
    integer :: tisr_size_input, tisr_size_res
    logical :: precip_bool, precip_input_bool
    integer :: precip_size_res, precip_size_input
    logical :: sst_bool, sst_bool_input, sst_bool_prediction
    integer :: sst_size_res, sst_size_input
    logical :: sst_climo_bool, sst_climo_input
    integer :: sst_climo_res
    logical :: atmo_to_ocean_coupled
    integer :: atmo_size_input, num_atmo_levels
    logical :: ohtc_input, ohtc_prediction
    integer :: ohtc_res_size, ohtc_input_size
    integer, allocatable :: atmo_training_data_idx(:)
    real(kind=dp), allocatable :: averaged_atmo_input_vec(:, :)
    integer :: chunk_size, chunk_size_prediction, chunk_size_speedy
    real(kind=dp), allocatable :: imperfect_model_states(:, :), predictiondata(:, :)
    real(kind=dp) :: noisemag, prior_val
    real(kind=dp), allocatable :: local_model(:), outvec(:), v_ml(:), v_p(:), feedback(:)
    real(kind=dp), allocatable :: full_tisr(:, :, :), full_sst(:, :, :)
    integer :: predictvars2d
  end type reservoir_type

  !> a NetCDF file kept open across reads (:624-631)
  type opened_netcdf_type
    logical :: is_opened, is_closed
    integer :: ncid
    character(len=:), allocatable :: filename
  end type opened_netcdf_type

  !> the run's static parameters (:369-505)
  type model_parameters_type
    logical :: ml_only, ml_only_ocean
    integer :: num_vert_levels, vert_loc_overlap, number_of_regions, num_of_regions_on_proc
    integer, allocatable :: region_indices(:)
    integer :: full_heightlevels, full_predictvars
    integer :: traininglength, discardlength, synclength, predictionlength, overlap
    integer, allocatable :: prediction_markers(:)
    integer :: num_predictions, current_trial_number
    integer :: irank, numprocs
    real(kind=dp), allocatable :: prediction(:, :)
    logical :: specific_humidity_log_bool
    real(kind=dp) :: specific_humidity_epsilon = 0.3_dp
    logical :: pole_only
    character(len=3) :: trial_number
    character(len=10) :: trial_date
    character(len=:), allocatable :: trial_name, trial_name_extra_end
    logical :: run_speedy, timeofday_bool, regional_vary, using_prior
    real(kind=dp) :: model_noise
    integer :: timestep, timestep_slab
    logical :: toa_isr_bool, precip_bool
    real :: precip_epsilon
    logical :: noisy
    character(len=:), allocatable :: prediction_file
    logical :: special_reservoirs
    integer :: num_special_reservoirs
    logical :: slab_ocean_model_bool, train_on_sst_anomalies
    real(kind=dp), allocatable :: base_sst_grid(:, :), sea_mask(:, :)
    type(opened_netcdf_type), allocatable :: opened_netcdf_files(:)
    logical :: non_stationary_ocn_climo
    real(kind=dp) :: final_sst_bias, current_sst_bias
    logical :: outvec_component_contribs
  end type model_parameters_type

  !> everything one rank holds (:507-532): grid(i,j) / reservoir(i,j) per local
  !> region i and vertical level j, the special (slab-ocean) ones, the parameters
  type main_type
    type(grid_type), allocatable :: grid(:, :)
    type(reservoir_type), allocatable :: reservoir(:, :)
    type(grid_type), allocatable :: grid_special(:, :)
    type(reservoir_type), allocatable :: reservoir_special(:, :)
    type(model_parameters_type) :: model_parameters
  end type main_type

  type speedy_data_type   ! :534-540
    real(kind=dp), allocatable :: speedyvariables(:, :, :, :, :), speedy_logp(:, :, :)
  end type speedy_data_type

  type era_data_type      ! :542-560
    real(kind=dp), allocatable :: eravariables(:, :, :, :, :), era_logp(:, :, :), era_tisr(:, :, :)
    real(kind=dp), allocatable :: era_sst(:, :, :), era_sst_climo(:, :, :), era_precip(:, :, :)
  end type era_data_type

  !> SPEEDY's grid state and start metadata handed to agcm_main (:562-591)
  type state_vector_type
    real(kind=dp), allocatable :: variables3d(:, :, :, :), logp(:, :)
    integer :: istart, era_start
    character(len=100) :: era_file
    integer :: era_hour, era_hour_plus_one
    integer :: iyear0, imont0, iday, ihour
    logical :: is_safe_to_run_speedy, hybrid_slab
    real(kind=dp), allocatable :: sst_hybrid(:, :)
    real(kind=dp) :: sst_bias = 0.0_dp
  end type state_vector_type

  !> the rank's place in the world (:593-604); with the GPU path the world is the
  !> RCCL communicator's (sml_comm_rank), mpi_world keeps the MPI handle's slot
  type mpi_type
    integer(kind=int32) :: ierr, numprocs, proc_num
    integer :: mpi_world
    logical :: is_root = .false.
    logical :: is_serial = .false.
  end type mpi_type

  type calendar_type      ! :606-622
    integer :: startyear, startmonth, startday, starthour
    integer :: currentyear, currentmonth, currentday, currenthour
  end type calendar_type
end module mod_utilities
