#include <stdio.h>
#include <string.h>
#include <stdbool.h>
#include <math.h>
#include <unistd.h>

#include "src/libs/canvas/canvas.h"
#include "src/libs/linalg/linalg.h"
#include "src/libs/obj_loader/obj_loader.h"
#include "src/libs/photon_map/pm.h"
#include "src/color/hsl.h"
#include "src/color/lab.h"
#include "src/color/rgb.h"
#include "src/color/srgb.h"
#include "src/color/xyz.h"
#include "src/color/xyy.h"

#include "src/renderer/camera.h"
#include "src/renderer/config.h"
#include "src/renderer/photon_tracer.h"
#include "src/renderer/renderer.h"
#include "src/renderer/world.h"
#include "src/pattern/pattern.h"
#include "src/shapes/shapes.h"
#include "src/shapes/cone.h"
#include "src/shapes/csg.h"
#include "src/shapes/cube.h"
#include "src/shapes/cylinder.h"
#include "src/shapes/group.h"
#include "src/shapes/plane.h"
#include "src/shapes/sphere.h"
#include "src/shapes/triangle.h"
#include "src/shapes/toroid.h"

#define True true
#define False false

int
main()
{
    /* config */
    struct global_config global_config;
    global_config.illumination.include_direct = True;
    global_config.illumination.include_global = False;
    global_config.illumination.debug_visualize_photon_map = False;
    global_config.illumination.debug_visualize_soft_indirect = False;
    global_config.illumination.di.include_ambient = True;
    global_config.illumination.di.include_diffuse = True;
    global_config.illumination.di.include_specular_highlight = True;
    global_config.illumination.di.include_specular = True;
    global_config.illumination.di.path_length = 5;

    global_config.illumination.gi.include_caustics = False;
    global_config.illumination.gi.include_final_gather = False;
    global_config.illumination.gi.usteps = 1;
    global_config.illumination.gi.vsteps = 1;
    global_config.illumination.gi.irradiance_estimate_num = 200;
    global_config.illumination.gi.irradiance_estimate_radius = 0.1000000000;
    global_config.illumination.gi.irradiance_estimate_cone_filter_k = 1.0000000000;
    global_config.illumination.gi.photon_count = 0;
    global_config.illumination.gi.path_length = 5;

    global_config.threading.num_threads = 8;
    global_config.scene.divide_threshold = 1;
    global_config.output.file_path = "/tmp/frt_golden/out/checkered_cube_160x80";
    global_config.output.color_space = SRGB;

    void (*color_space_fn)(const Color, Color) = NULL;
    switch (global_config.output.color_space) {
    case RGB:
        color_space_fn = rgb_to_rgb;
        break;
    case HSL:
        color_space_fn = hsl_to_rgb;
        break;
    case XYZ:
        color_space_fn = xyz_to_rgb;
        break;
    case XYY:
        color_space_fn = xyy_to_rgb;
        break;
    case LAB:
        color_space_fn = lab_to_rgb;
        break;
    case SRGB:
        // this is the default
    default:
        color_space_fn = srgb_to_rgb;
        break;
    }

    /* end config */

    /* camera */
    struct aperture ap;
    aperture(POINT_APERTURE, 0.0, 1, 1, false, &ap);

    Point from = { 0.0000000000, 0.0000000000, -20.0000000000, 1.0 };
    Point to = { 0.0000000000, 0.0000000000, 0.0000000000, 1.0 };
    Vector up = { 0.0000000000, 1.0000000000, 0.0000000000, 0.0 };
    Matrix camera_xform;
    view_transform(from, to, up, camera_xform);

    Camera cam = camera(160, 80, 0.8000000000/*field_of_view*/, 1.0000000000/*distance*/, 1/*usteps*/, 1/*vsteps*/, &ap, camera_xform);

    /* end camera */

    /* lights */
    Light all_lights = array_of_lights(4);

    /* point light 0 */
    Light point_light_0 = all_lights + 0;
    Point point_light_0_point = { 0.0000000000, 100.0000000000, -100.0000000000, 1.0 };
    Color point_light_0_intensity = color(0.2500000000, 0.2500000000, 0.2500000000);
    point_light(point_light_0_point, point_light_0_intensity, point_light_0);

    /* end point light 0 */
    /* point light 1 */
    Light point_light_1 = all_lights + 1;
    Point point_light_1_point = { 0.0000000000, -100.0000000000, -100.0000000000, 1.0 };
    Color point_light_1_intensity = color(0.2500000000, 0.2500000000, 0.2500000000);
    point_light(point_light_1_point, point_light_1_intensity, point_light_1);

    /* end point light 1 */
    /* point light 2 */
    Light point_light_2 = all_lights + 2;
    Point point_light_2_point = { -100.0000000000, 0.0000000000, -100.0000000000, 1.0 };
    Color point_light_2_intensity = color(0.2500000000, 0.2500000000, 0.2500000000);
    point_light(point_light_2_point, point_light_2_intensity, point_light_2);

    /* end point light 2 */
    /* point light 3 */
    Light point_light_3 = all_lights + 3;
    Point point_light_3_point = { 100.0000000000, 0.0000000000, -100.0000000000, 1.0 };
    Color point_light_3_intensity = color(0.2500000000, 0.2500000000, 0.2500000000);
    point_light(point_light_3_point, point_light_3_intensity, point_light_3);

    /* end point light 3 */

    /* end lights */

    /* shapes */
    Shape all_shapes = array_of_shapes(8);

    /* shape 0 */
    
    Matrix transform_pattern_0_Ka;
    matrix_identity(transform_pattern_0_Ka);
    Pattern pattern_0_Ka = array_of_patterns(7);
    Pattern pattern_0_Ka_right = pattern_0_Ka + 1;
    Pattern pattern_0_Ka_left = pattern_0_Ka + 2;
    Pattern pattern_0_Ka_up = pattern_0_Ka + 3;
    Pattern pattern_0_Ka_down = pattern_0_Ka + 4;
    Pattern pattern_0_Ka_front = pattern_0_Ka + 5;
    Pattern pattern_0_Ka_back = pattern_0_Ka + 6;

    Color pattern_0_Ka_right_color_0_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_0_Ka_right_color_1_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_0_Ka_right_color_2_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_0_Ka_right_color_3_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_0_Ka_right_color_4_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_0_Ka_right_color_0;
    Color pattern_0_Ka_right_color_1;
    Color pattern_0_Ka_right_color_2;
    Color pattern_0_Ka_right_color_3;
    Color pattern_0_Ka_right_color_4;
    color_space_fn(pattern_0_Ka_right_color_0_raw, pattern_0_Ka_right_color_0);
    color_space_fn(pattern_0_Ka_right_color_1_raw, pattern_0_Ka_right_color_1);
    color_space_fn(pattern_0_Ka_right_color_2_raw, pattern_0_Ka_right_color_2);
    color_space_fn(pattern_0_Ka_right_color_3_raw, pattern_0_Ka_right_color_3);
    color_space_fn(pattern_0_Ka_right_color_4_raw, pattern_0_Ka_right_color_4);
    uv_align_check_pattern(pattern_0_Ka_right_color_0, pattern_0_Ka_right_color_1, pattern_0_Ka_right_color_2, pattern_0_Ka_right_color_3, pattern_0_Ka_right_color_4, pattern_0_Ka_right);


    Color pattern_0_Ka_left_color_0_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_0_Ka_left_color_1_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_0_Ka_left_color_2_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_0_Ka_left_color_3_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_0_Ka_left_color_4_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_0_Ka_left_color_0;
    Color pattern_0_Ka_left_color_1;
    Color pattern_0_Ka_left_color_2;
    Color pattern_0_Ka_left_color_3;
    Color pattern_0_Ka_left_color_4;
    color_space_fn(pattern_0_Ka_left_color_0_raw, pattern_0_Ka_left_color_0);
    color_space_fn(pattern_0_Ka_left_color_1_raw, pattern_0_Ka_left_color_1);
    color_space_fn(pattern_0_Ka_left_color_2_raw, pattern_0_Ka_left_color_2);
    color_space_fn(pattern_0_Ka_left_color_3_raw, pattern_0_Ka_left_color_3);
    color_space_fn(pattern_0_Ka_left_color_4_raw, pattern_0_Ka_left_color_4);
    uv_align_check_pattern(pattern_0_Ka_left_color_0, pattern_0_Ka_left_color_1, pattern_0_Ka_left_color_2, pattern_0_Ka_left_color_3, pattern_0_Ka_left_color_4, pattern_0_Ka_left);


    Color pattern_0_Ka_up_color_0_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_0_Ka_up_color_1_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_0_Ka_up_color_2_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_0_Ka_up_color_3_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_0_Ka_up_color_4_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_0_Ka_up_color_0;
    Color pattern_0_Ka_up_color_1;
    Color pattern_0_Ka_up_color_2;
    Color pattern_0_Ka_up_color_3;
    Color pattern_0_Ka_up_color_4;
    color_space_fn(pattern_0_Ka_up_color_0_raw, pattern_0_Ka_up_color_0);
    color_space_fn(pattern_0_Ka_up_color_1_raw, pattern_0_Ka_up_color_1);
    color_space_fn(pattern_0_Ka_up_color_2_raw, pattern_0_Ka_up_color_2);
    color_space_fn(pattern_0_Ka_up_color_3_raw, pattern_0_Ka_up_color_3);
    color_space_fn(pattern_0_Ka_up_color_4_raw, pattern_0_Ka_up_color_4);
    uv_align_check_pattern(pattern_0_Ka_up_color_0, pattern_0_Ka_up_color_1, pattern_0_Ka_up_color_2, pattern_0_Ka_up_color_3, pattern_0_Ka_up_color_4, pattern_0_Ka_up);


    Color pattern_0_Ka_down_color_0_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_0_Ka_down_color_1_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_0_Ka_down_color_2_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_0_Ka_down_color_3_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_0_Ka_down_color_4_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_0_Ka_down_color_0;
    Color pattern_0_Ka_down_color_1;
    Color pattern_0_Ka_down_color_2;
    Color pattern_0_Ka_down_color_3;
    Color pattern_0_Ka_down_color_4;
    color_space_fn(pattern_0_Ka_down_color_0_raw, pattern_0_Ka_down_color_0);
    color_space_fn(pattern_0_Ka_down_color_1_raw, pattern_0_Ka_down_color_1);
    color_space_fn(pattern_0_Ka_down_color_2_raw, pattern_0_Ka_down_color_2);
    color_space_fn(pattern_0_Ka_down_color_3_raw, pattern_0_Ka_down_color_3);
    color_space_fn(pattern_0_Ka_down_color_4_raw, pattern_0_Ka_down_color_4);
    uv_align_check_pattern(pattern_0_Ka_down_color_0, pattern_0_Ka_down_color_1, pattern_0_Ka_down_color_2, pattern_0_Ka_down_color_3, pattern_0_Ka_down_color_4, pattern_0_Ka_down);


    Color pattern_0_Ka_front_color_0_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_0_Ka_front_color_1_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_0_Ka_front_color_2_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_0_Ka_front_color_3_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_0_Ka_front_color_4_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_0_Ka_front_color_0;
    Color pattern_0_Ka_front_color_1;
    Color pattern_0_Ka_front_color_2;
    Color pattern_0_Ka_front_color_3;
    Color pattern_0_Ka_front_color_4;
    color_space_fn(pattern_0_Ka_front_color_0_raw, pattern_0_Ka_front_color_0);
    color_space_fn(pattern_0_Ka_front_color_1_raw, pattern_0_Ka_front_color_1);
    color_space_fn(pattern_0_Ka_front_color_2_raw, pattern_0_Ka_front_color_2);
    color_space_fn(pattern_0_Ka_front_color_3_raw, pattern_0_Ka_front_color_3);
    color_space_fn(pattern_0_Ka_front_color_4_raw, pattern_0_Ka_front_color_4);
    uv_align_check_pattern(pattern_0_Ka_front_color_0, pattern_0_Ka_front_color_1, pattern_0_Ka_front_color_2, pattern_0_Ka_front_color_3, pattern_0_Ka_front_color_4, pattern_0_Ka_front);


    Color pattern_0_Ka_back_color_0_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_0_Ka_back_color_1_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_0_Ka_back_color_2_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_0_Ka_back_color_3_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_0_Ka_back_color_4_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_0_Ka_back_color_0;
    Color pattern_0_Ka_back_color_1;
    Color pattern_0_Ka_back_color_2;
    Color pattern_0_Ka_back_color_3;
    Color pattern_0_Ka_back_color_4;
    color_space_fn(pattern_0_Ka_back_color_0_raw, pattern_0_Ka_back_color_0);
    color_space_fn(pattern_0_Ka_back_color_1_raw, pattern_0_Ka_back_color_1);
    color_space_fn(pattern_0_Ka_back_color_2_raw, pattern_0_Ka_back_color_2);
    color_space_fn(pattern_0_Ka_back_color_3_raw, pattern_0_Ka_back_color_3);
    color_space_fn(pattern_0_Ka_back_color_4_raw, pattern_0_Ka_back_color_4);
    uv_align_check_pattern(pattern_0_Ka_back_color_0, pattern_0_Ka_back_color_1, pattern_0_Ka_back_color_2, pattern_0_Ka_back_color_3, pattern_0_Ka_back_color_4, pattern_0_Ka_back);



    texture_map_pattern(pattern_0_Ka_right, CUBE_UV_MAP, pattern_0_Ka);
    pattern_set_transform(pattern_0_Ka, transform_pattern_0_Ka);
Matrix transform_pattern_0_Kd;
    matrix_identity(transform_pattern_0_Kd);
    Pattern pattern_0_Kd = array_of_patterns(7);
    Pattern pattern_0_Kd_right = pattern_0_Kd + 1;
    Pattern pattern_0_Kd_left = pattern_0_Kd + 2;
    Pattern pattern_0_Kd_up = pattern_0_Kd + 3;
    Pattern pattern_0_Kd_down = pattern_0_Kd + 4;
    Pattern pattern_0_Kd_front = pattern_0_Kd + 5;
    Pattern pattern_0_Kd_back = pattern_0_Kd + 6;

    Color pattern_0_Kd_right_color_0_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_0_Kd_right_color_1_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_0_Kd_right_color_2_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_0_Kd_right_color_3_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_0_Kd_right_color_4_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_0_Kd_right_color_0;
    Color pattern_0_Kd_right_color_1;
    Color pattern_0_Kd_right_color_2;
    Color pattern_0_Kd_right_color_3;
    Color pattern_0_Kd_right_color_4;
    color_space_fn(pattern_0_Kd_right_color_0_raw, pattern_0_Kd_right_color_0);
    color_space_fn(pattern_0_Kd_right_color_1_raw, pattern_0_Kd_right_color_1);
    color_space_fn(pattern_0_Kd_right_color_2_raw, pattern_0_Kd_right_color_2);
    color_space_fn(pattern_0_Kd_right_color_3_raw, pattern_0_Kd_right_color_3);
    color_space_fn(pattern_0_Kd_right_color_4_raw, pattern_0_Kd_right_color_4);
    uv_align_check_pattern(pattern_0_Kd_right_color_0, pattern_0_Kd_right_color_1, pattern_0_Kd_right_color_2, pattern_0_Kd_right_color_3, pattern_0_Kd_right_color_4, pattern_0_Kd_right);


    Color pattern_0_Kd_left_color_0_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_0_Kd_left_color_1_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_0_Kd_left_color_2_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_0_Kd_left_color_3_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_0_Kd_left_color_4_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_0_Kd_left_color_0;
    Color pattern_0_Kd_left_color_1;
    Color pattern_0_Kd_left_color_2;
    Color pattern_0_Kd_left_color_3;
    Color pattern_0_Kd_left_color_4;
    color_space_fn(pattern_0_Kd_left_color_0_raw, pattern_0_Kd_left_color_0);
    color_space_fn(pattern_0_Kd_left_color_1_raw, pattern_0_Kd_left_color_1);
    color_space_fn(pattern_0_Kd_left_color_2_raw, pattern_0_Kd_left_color_2);
    color_space_fn(pattern_0_Kd_left_color_3_raw, pattern_0_Kd_left_color_3);
    color_space_fn(pattern_0_Kd_left_color_4_raw, pattern_0_Kd_left_color_4);
    uv_align_check_pattern(pattern_0_Kd_left_color_0, pattern_0_Kd_left_color_1, pattern_0_Kd_left_color_2, pattern_0_Kd_left_color_3, pattern_0_Kd_left_color_4, pattern_0_Kd_left);


    Color pattern_0_Kd_up_color_0_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_0_Kd_up_color_1_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_0_Kd_up_color_2_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_0_Kd_up_color_3_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_0_Kd_up_color_4_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_0_Kd_up_color_0;
    Color pattern_0_Kd_up_color_1;
    Color pattern_0_Kd_up_color_2;
    Color pattern_0_Kd_up_color_3;
    Color pattern_0_Kd_up_color_4;
    color_space_fn(pattern_0_Kd_up_color_0_raw, pattern_0_Kd_up_color_0);
    color_space_fn(pattern_0_Kd_up_color_1_raw, pattern_0_Kd_up_color_1);
    color_space_fn(pattern_0_Kd_up_color_2_raw, pattern_0_Kd_up_color_2);
    color_space_fn(pattern_0_Kd_up_color_3_raw, pattern_0_Kd_up_color_3);
    color_space_fn(pattern_0_Kd_up_color_4_raw, pattern_0_Kd_up_color_4);
    uv_align_check_pattern(pattern_0_Kd_up_color_0, pattern_0_Kd_up_color_1, pattern_0_Kd_up_color_2, pattern_0_Kd_up_color_3, pattern_0_Kd_up_color_4, pattern_0_Kd_up);


    Color pattern_0_Kd_down_color_0_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_0_Kd_down_color_1_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_0_Kd_down_color_2_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_0_Kd_down_color_3_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_0_Kd_down_color_4_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_0_Kd_down_color_0;
    Color pattern_0_Kd_down_color_1;
    Color pattern_0_Kd_down_color_2;
    Color pattern_0_Kd_down_color_3;
    Color pattern_0_Kd_down_color_4;
    color_space_fn(pattern_0_Kd_down_color_0_raw, pattern_0_Kd_down_color_0);
    color_space_fn(pattern_0_Kd_down_color_1_raw, pattern_0_Kd_down_color_1);
    color_space_fn(pattern_0_Kd_down_color_2_raw, pattern_0_Kd_down_color_2);
    color_space_fn(pattern_0_Kd_down_color_3_raw, pattern_0_Kd_down_color_3);
    color_space_fn(pattern_0_Kd_down_color_4_raw, pattern_0_Kd_down_color_4);
    uv_align_check_pattern(pattern_0_Kd_down_color_0, pattern_0_Kd_down_color_1, pattern_0_Kd_down_color_2, pattern_0_Kd_down_color_3, pattern_0_Kd_down_color_4, pattern_0_Kd_down);


    Color pattern_0_Kd_front_color_0_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_0_Kd_front_color_1_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_0_Kd_front_color_2_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_0_Kd_front_color_3_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_0_Kd_front_color_4_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_0_Kd_front_color_0;
    Color pattern_0_Kd_front_color_1;
    Color pattern_0_Kd_front_color_2;
    Color pattern_0_Kd_front_color_3;
    Color pattern_0_Kd_front_color_4;
    color_space_fn(pattern_0_Kd_front_color_0_raw, pattern_0_Kd_front_color_0);
    color_space_fn(pattern_0_Kd_front_color_1_raw, pattern_0_Kd_front_color_1);
    color_space_fn(pattern_0_Kd_front_color_2_raw, pattern_0_Kd_front_color_2);
    color_space_fn(pattern_0_Kd_front_color_3_raw, pattern_0_Kd_front_color_3);
    color_space_fn(pattern_0_Kd_front_color_4_raw, pattern_0_Kd_front_color_4);
    uv_align_check_pattern(pattern_0_Kd_front_color_0, pattern_0_Kd_front_color_1, pattern_0_Kd_front_color_2, pattern_0_Kd_front_color_3, pattern_0_Kd_front_color_4, pattern_0_Kd_front);


    Color pattern_0_Kd_back_color_0_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_0_Kd_back_color_1_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_0_Kd_back_color_2_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_0_Kd_back_color_3_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_0_Kd_back_color_4_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_0_Kd_back_color_0;
    Color pattern_0_Kd_back_color_1;
    Color pattern_0_Kd_back_color_2;
    Color pattern_0_Kd_back_color_3;
    Color pattern_0_Kd_back_color_4;
    color_space_fn(pattern_0_Kd_back_color_0_raw, pattern_0_Kd_back_color_0);
    color_space_fn(pattern_0_Kd_back_color_1_raw, pattern_0_Kd_back_color_1);
    color_space_fn(pattern_0_Kd_back_color_2_raw, pattern_0_Kd_back_color_2);
    color_space_fn(pattern_0_Kd_back_color_3_raw, pattern_0_Kd_back_color_3);
    color_space_fn(pattern_0_Kd_back_color_4_raw, pattern_0_Kd_back_color_4);
    uv_align_check_pattern(pattern_0_Kd_back_color_0, pattern_0_Kd_back_color_1, pattern_0_Kd_back_color_2, pattern_0_Kd_back_color_3, pattern_0_Kd_back_color_4, pattern_0_Kd_back);



    texture_map_pattern(pattern_0_Kd_right, CUBE_UV_MAP, pattern_0_Kd);
    pattern_set_transform(pattern_0_Kd, transform_pattern_0_Kd);
    Pattern pattern_0_Ks = NULL;
    Pattern pattern_0_Ns = NULL;
    Pattern pattern_0_bump = NULL;
    Pattern pattern_0_disp = NULL;
    Pattern pattern_0_refl = NULL;
    Pattern pattern_0_d = NULL;
    Color material_0_color_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color material_0_reflective = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_0_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_0 = material_alloc();
    color_space_fn(material_0_color_raw, material_0->Ka);
    color_space_fn(material_0_color_raw, material_0->Kd);
    color_space_fn(material_0_color_raw, material_0->Ks);
    color_scale(material_0->Ka, 0.2000000000);
    color_scale(material_0->Kd, 0.8000000000);
    color_scale(material_0->Ks, 0.0000000000);
    rgb_to_rgb(material_0_reflective, material_0->refl);
    rgb_to_rgb(material_0_refractive, material_0->Tf);
    material_0->reflective = material_0_reflective[0] > 0.0
                             || material_0_reflective[1] > 0.0
                             || material_0_reflective[2] > 0.0;

    material_0->Tr = 0.0000000000;
    material_0->Ns = 200.0000000000;
    material_0->Ni = 1.0000000000;
    material_0->casts_shadow = true;
    material_set_pattern(material_0, map_Ka, pattern_0_Ka);
    material_set_pattern(material_0, map_Kd, pattern_0_Kd);
    material_set_pattern(material_0, map_Ks, pattern_0_Ks);
    material_set_pattern(material_0, map_Ns, pattern_0_Ns);
    material_set_pattern(material_0, map_d, pattern_0_d);
    material_set_pattern(material_0, map_bump, pattern_0_bump);
    material_set_pattern(material_0, map_disp, pattern_0_disp);
    material_set_pattern(material_0, map_refl, pattern_0_refl);

    Matrix transform_0, transform_0_tmp;
    matrix_identity(transform_0);
    matrix_rotate_y(0.7854000000, transform_0_tmp);
    transform_chain(transform_0_tmp, transform_0);
    matrix_rotate_x(0.7854000000, transform_0_tmp);
    transform_chain(transform_0_tmp, transform_0);
    matrix_translate(-6.0000000000, 2.0000000000, 0.0000000000, transform_0_tmp);
    transform_chain(transform_0_tmp, transform_0);

    Shape shape_0 = all_shapes + 0;
    cube(shape_0);
    shape_set_material(shape_0, material_0);
    shape_set_transform(shape_0, transform_0);

    /* end shape 0 */
    /* shape 1 */
    
    Matrix transform_pattern_1_Ka;
    matrix_identity(transform_pattern_1_Ka);
    Pattern pattern_1_Ka = array_of_patterns(7);
    Pattern pattern_1_Ka_right = pattern_1_Ka + 1;
    Pattern pattern_1_Ka_left = pattern_1_Ka + 2;
    Pattern pattern_1_Ka_up = pattern_1_Ka + 3;
    Pattern pattern_1_Ka_down = pattern_1_Ka + 4;
    Pattern pattern_1_Ka_front = pattern_1_Ka + 5;
    Pattern pattern_1_Ka_back = pattern_1_Ka + 6;

    Color pattern_1_Ka_right_color_0_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_1_Ka_right_color_1_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_1_Ka_right_color_2_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_1_Ka_right_color_3_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_1_Ka_right_color_4_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_1_Ka_right_color_0;
    Color pattern_1_Ka_right_color_1;
    Color pattern_1_Ka_right_color_2;
    Color pattern_1_Ka_right_color_3;
    Color pattern_1_Ka_right_color_4;
    color_space_fn(pattern_1_Ka_right_color_0_raw, pattern_1_Ka_right_color_0);
    color_space_fn(pattern_1_Ka_right_color_1_raw, pattern_1_Ka_right_color_1);
    color_space_fn(pattern_1_Ka_right_color_2_raw, pattern_1_Ka_right_color_2);
    color_space_fn(pattern_1_Ka_right_color_3_raw, pattern_1_Ka_right_color_3);
    color_space_fn(pattern_1_Ka_right_color_4_raw, pattern_1_Ka_right_color_4);
    uv_align_check_pattern(pattern_1_Ka_right_color_0, pattern_1_Ka_right_color_1, pattern_1_Ka_right_color_2, pattern_1_Ka_right_color_3, pattern_1_Ka_right_color_4, pattern_1_Ka_right);


    Color pattern_1_Ka_left_color_0_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_1_Ka_left_color_1_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_1_Ka_left_color_2_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_1_Ka_left_color_3_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_1_Ka_left_color_4_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_1_Ka_left_color_0;
    Color pattern_1_Ka_left_color_1;
    Color pattern_1_Ka_left_color_2;
    Color pattern_1_Ka_left_color_3;
    Color pattern_1_Ka_left_color_4;
    color_space_fn(pattern_1_Ka_left_color_0_raw, pattern_1_Ka_left_color_0);
    color_space_fn(pattern_1_Ka_left_color_1_raw, pattern_1_Ka_left_color_1);
    color_space_fn(pattern_1_Ka_left_color_2_raw, pattern_1_Ka_left_color_2);
    color_space_fn(pattern_1_Ka_left_color_3_raw, pattern_1_Ka_left_color_3);
    color_space_fn(pattern_1_Ka_left_color_4_raw, pattern_1_Ka_left_color_4);
    uv_align_check_pattern(pattern_1_Ka_left_color_0, pattern_1_Ka_left_color_1, pattern_1_Ka_left_color_2, pattern_1_Ka_left_color_3, pattern_1_Ka_left_color_4, pattern_1_Ka_left);


    Color pattern_1_Ka_up_color_0_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_1_Ka_up_color_1_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_1_Ka_up_color_2_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_1_Ka_up_color_3_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_1_Ka_up_color_4_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_1_Ka_up_color_0;
    Color pattern_1_Ka_up_color_1;
    Color pattern_1_Ka_up_color_2;
    Color pattern_1_Ka_up_color_3;
    Color pattern_1_Ka_up_color_4;
    color_space_fn(pattern_1_Ka_up_color_0_raw, pattern_1_Ka_up_color_0);
    color_space_fn(pattern_1_Ka_up_color_1_raw, pattern_1_Ka_up_color_1);
    color_space_fn(pattern_1_Ka_up_color_2_raw, pattern_1_Ka_up_color_2);
    color_space_fn(pattern_1_Ka_up_color_3_raw, pattern_1_Ka_up_color_3);
    color_space_fn(pattern_1_Ka_up_color_4_raw, pattern_1_Ka_up_color_4);
    uv_align_check_pattern(pattern_1_Ka_up_color_0, pattern_1_Ka_up_color_1, pattern_1_Ka_up_color_2, pattern_1_Ka_up_color_3, pattern_1_Ka_up_color_4, pattern_1_Ka_up);


    Color pattern_1_Ka_down_color_0_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_1_Ka_down_color_1_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_1_Ka_down_color_2_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_1_Ka_down_color_3_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_1_Ka_down_color_4_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_1_Ka_down_color_0;
    Color pattern_1_Ka_down_color_1;
    Color pattern_1_Ka_down_color_2;
    Color pattern_1_Ka_down_color_3;
    Color pattern_1_Ka_down_color_4;
    color_space_fn(pattern_1_Ka_down_color_0_raw, pattern_1_Ka_down_color_0);
    color_space_fn(pattern_1_Ka_down_color_1_raw, pattern_1_Ka_down_color_1);
    color_space_fn(pattern_1_Ka_down_color_2_raw, pattern_1_Ka_down_color_2);
    color_space_fn(pattern_1_Ka_down_color_3_raw, pattern_1_Ka_down_color_3);
    color_space_fn(pattern_1_Ka_down_color_4_raw, pattern_1_Ka_down_color_4);
    uv_align_check_pattern(pattern_1_Ka_down_color_0, pattern_1_Ka_down_color_1, pattern_1_Ka_down_color_2, pattern_1_Ka_down_color_3, pattern_1_Ka_down_color_4, pattern_1_Ka_down);


    Color pattern_1_Ka_front_color_0_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_1_Ka_front_color_1_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_1_Ka_front_color_2_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_1_Ka_front_color_3_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_1_Ka_front_color_4_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_1_Ka_front_color_0;
    Color pattern_1_Ka_front_color_1;
    Color pattern_1_Ka_front_color_2;
    Color pattern_1_Ka_front_color_3;
    Color pattern_1_Ka_front_color_4;
    color_space_fn(pattern_1_Ka_front_color_0_raw, pattern_1_Ka_front_color_0);
    color_space_fn(pattern_1_Ka_front_color_1_raw, pattern_1_Ka_front_color_1);
    color_space_fn(pattern_1_Ka_front_color_2_raw, pattern_1_Ka_front_color_2);
    color_space_fn(pattern_1_Ka_front_color_3_raw, pattern_1_Ka_front_color_3);
    color_space_fn(pattern_1_Ka_front_color_4_raw, pattern_1_Ka_front_color_4);
    uv_align_check_pattern(pattern_1_Ka_front_color_0, pattern_1_Ka_front_color_1, pattern_1_Ka_front_color_2, pattern_1_Ka_front_color_3, pattern_1_Ka_front_color_4, pattern_1_Ka_front);


    Color pattern_1_Ka_back_color_0_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_1_Ka_back_color_1_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_1_Ka_back_color_2_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_1_Ka_back_color_3_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_1_Ka_back_color_4_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_1_Ka_back_color_0;
    Color pattern_1_Ka_back_color_1;
    Color pattern_1_Ka_back_color_2;
    Color pattern_1_Ka_back_color_3;
    Color pattern_1_Ka_back_color_4;
    color_space_fn(pattern_1_Ka_back_color_0_raw, pattern_1_Ka_back_color_0);
    color_space_fn(pattern_1_Ka_back_color_1_raw, pattern_1_Ka_back_color_1);
    color_space_fn(pattern_1_Ka_back_color_2_raw, pattern_1_Ka_back_color_2);
    color_space_fn(pattern_1_Ka_back_color_3_raw, pattern_1_Ka_back_color_3);
    color_space_fn(pattern_1_Ka_back_color_4_raw, pattern_1_Ka_back_color_4);
    uv_align_check_pattern(pattern_1_Ka_back_color_0, pattern_1_Ka_back_color_1, pattern_1_Ka_back_color_2, pattern_1_Ka_back_color_3, pattern_1_Ka_back_color_4, pattern_1_Ka_back);



    texture_map_pattern(pattern_1_Ka_right, CUBE_UV_MAP, pattern_1_Ka);
    pattern_set_transform(pattern_1_Ka, transform_pattern_1_Ka);
Matrix transform_pattern_1_Kd;
    matrix_identity(transform_pattern_1_Kd);
    Pattern pattern_1_Kd = array_of_patterns(7);
    Pattern pattern_1_Kd_right = pattern_1_Kd + 1;
    Pattern pattern_1_Kd_left = pattern_1_Kd + 2;
    Pattern pattern_1_Kd_up = pattern_1_Kd + 3;
    Pattern pattern_1_Kd_down = pattern_1_Kd + 4;
    Pattern pattern_1_Kd_front = pattern_1_Kd + 5;
    Pattern pattern_1_Kd_back = pattern_1_Kd + 6;

    Color pattern_1_Kd_right_color_0_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_1_Kd_right_color_1_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_1_Kd_right_color_2_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_1_Kd_right_color_3_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_1_Kd_right_color_4_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_1_Kd_right_color_0;
    Color pattern_1_Kd_right_color_1;
    Color pattern_1_Kd_right_color_2;
    Color pattern_1_Kd_right_color_3;
    Color pattern_1_Kd_right_color_4;
    color_space_fn(pattern_1_Kd_right_color_0_raw, pattern_1_Kd_right_color_0);
    color_space_fn(pattern_1_Kd_right_color_1_raw, pattern_1_Kd_right_color_1);
    color_space_fn(pattern_1_Kd_right_color_2_raw, pattern_1_Kd_right_color_2);
    color_space_fn(pattern_1_Kd_right_color_3_raw, pattern_1_Kd_right_color_3);
    color_space_fn(pattern_1_Kd_right_color_4_raw, pattern_1_Kd_right_color_4);
    uv_align_check_pattern(pattern_1_Kd_right_color_0, pattern_1_Kd_right_color_1, pattern_1_Kd_right_color_2, pattern_1_Kd_right_color_3, pattern_1_Kd_right_color_4, pattern_1_Kd_right);


    Color pattern_1_Kd_left_color_0_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_1_Kd_left_color_1_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_1_Kd_left_color_2_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_1_Kd_left_color_3_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_1_Kd_left_color_4_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_1_Kd_left_color_0;
    Color pattern_1_Kd_left_color_1;
    Color pattern_1_Kd_left_color_2;
    Color pattern_1_Kd_left_color_3;
    Color pattern_1_Kd_left_color_4;
    color_space_fn(pattern_1_Kd_left_color_0_raw, pattern_1_Kd_left_color_0);
    color_space_fn(pattern_1_Kd_left_color_1_raw, pattern_1_Kd_left_color_1);
    color_space_fn(pattern_1_Kd_left_color_2_raw, pattern_1_Kd_left_color_2);
    color_space_fn(pattern_1_Kd_left_color_3_raw, pattern_1_Kd_left_color_3);
    color_space_fn(pattern_1_Kd_left_color_4_raw, pattern_1_Kd_left_color_4);
    uv_align_check_pattern(pattern_1_Kd_left_color_0, pattern_1_Kd_left_color_1, pattern_1_Kd_left_color_2, pattern_1_Kd_left_color_3, pattern_1_Kd_left_color_4, pattern_1_Kd_left);


    Color pattern_1_Kd_up_color_0_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_1_Kd_up_color_1_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_1_Kd_up_color_2_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_1_Kd_up_color_3_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_1_Kd_up_color_4_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_1_Kd_up_color_0;
    Color pattern_1_Kd_up_color_1;
    Color pattern_1_Kd_up_color_2;
    Color pattern_1_Kd_up_color_3;
    Color pattern_1_Kd_up_color_4;
    color_space_fn(pattern_1_Kd_up_color_0_raw, pattern_1_Kd_up_color_0);
    color_space_fn(pattern_1_Kd_up_color_1_raw, pattern_1_Kd_up_color_1);
    color_space_fn(pattern_1_Kd_up_color_2_raw, pattern_1_Kd_up_color_2);
    color_space_fn(pattern_1_Kd_up_color_3_raw, pattern_1_Kd_up_color_3);
    color_space_fn(pattern_1_Kd_up_color_4_raw, pattern_1_Kd_up_color_4);
    uv_align_check_pattern(pattern_1_Kd_up_color_0, pattern_1_Kd_up_color_1, pattern_1_Kd_up_color_2, pattern_1_Kd_up_color_3, pattern_1_Kd_up_color_4, pattern_1_Kd_up);


    Color pattern_1_Kd_down_color_0_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_1_Kd_down_color_1_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_1_Kd_down_color_2_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_1_Kd_down_color_3_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_1_Kd_down_color_4_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_1_Kd_down_color_0;
    Color pattern_1_Kd_down_color_1;
    Color pattern_1_Kd_down_color_2;
    Color pattern_1_Kd_down_color_3;
    Color pattern_1_Kd_down_color_4;
    color_space_fn(pattern_1_Kd_down_color_0_raw, pattern_1_Kd_down_color_0);
    color_space_fn(pattern_1_Kd_down_color_1_raw, pattern_1_Kd_down_color_1);
    color_space_fn(pattern_1_Kd_down_color_2_raw, pattern_1_Kd_down_color_2);
    color_space_fn(pattern_1_Kd_down_color_3_raw, pattern_1_Kd_down_color_3);
    color_space_fn(pattern_1_Kd_down_color_4_raw, pattern_1_Kd_down_color_4);
    uv_align_check_pattern(pattern_1_Kd_down_color_0, pattern_1_Kd_down_color_1, pattern_1_Kd_down_color_2, pattern_1_Kd_down_color_3, pattern_1_Kd_down_color_4, pattern_1_Kd_down);


    Color pattern_1_Kd_front_color_0_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_1_Kd_front_color_1_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_1_Kd_front_color_2_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_1_Kd_front_color_3_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_1_Kd_front_color_4_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_1_Kd_front_color_0;
    Color pattern_1_Kd_front_color_1;
    Color pattern_1_Kd_front_color_2;
    Color pattern_1_Kd_front_color_3;
    Color pattern_1_Kd_front_color_4;
    color_space_fn(pattern_1_Kd_front_color_0_raw, pattern_1_Kd_front_color_0);
    color_space_fn(pattern_1_Kd_front_color_1_raw, pattern_1_Kd_front_color_1);
    color_space_fn(pattern_1_Kd_front_color_2_raw, pattern_1_Kd_front_color_2);
    color_space_fn(pattern_1_Kd_front_color_3_raw, pattern_1_Kd_front_color_3);
    color_space_fn(pattern_1_Kd_front_color_4_raw, pattern_1_Kd_front_color_4);
    uv_align_check_pattern(pattern_1_Kd_front_color_0, pattern_1_Kd_front_color_1, pattern_1_Kd_front_color_2, pattern_1_Kd_front_color_3, pattern_1_Kd_front_color_4, pattern_1_Kd_front);


    Color pattern_1_Kd_back_color_0_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_1_Kd_back_color_1_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_1_Kd_back_color_2_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_1_Kd_back_color_3_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_1_Kd_back_color_4_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_1_Kd_back_color_0;
    Color pattern_1_Kd_back_color_1;
    Color pattern_1_Kd_back_color_2;
    Color pattern_1_Kd_back_color_3;
    Color pattern_1_Kd_back_color_4;
    color_space_fn(pattern_1_Kd_back_color_0_raw, pattern_1_Kd_back_color_0);
    color_space_fn(pattern_1_Kd_back_color_1_raw, pattern_1_Kd_back_color_1);
    color_space_fn(pattern_1_Kd_back_color_2_raw, pattern_1_Kd_back_color_2);
    color_space_fn(pattern_1_Kd_back_color_3_raw, pattern_1_Kd_back_color_3);
    color_space_fn(pattern_1_Kd_back_color_4_raw, pattern_1_Kd_back_color_4);
    uv_align_check_pattern(pattern_1_Kd_back_color_0, pattern_1_Kd_back_color_1, pattern_1_Kd_back_color_2, pattern_1_Kd_back_color_3, pattern_1_Kd_back_color_4, pattern_1_Kd_back);



    texture_map_pattern(pattern_1_Kd_right, CUBE_UV_MAP, pattern_1_Kd);
    pattern_set_transform(pattern_1_Kd, transform_pattern_1_Kd);
    Pattern pattern_1_Ks = NULL;
    Pattern pattern_1_Ns = NULL;
    Pattern pattern_1_bump = NULL;
    Pattern pattern_1_disp = NULL;
    Pattern pattern_1_refl = NULL;
    Pattern pattern_1_d = NULL;
    Color material_1_color_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color material_1_reflective = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_1_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_1 = material_alloc();
    color_space_fn(material_1_color_raw, material_1->Ka);
    color_space_fn(material_1_color_raw, material_1->Kd);
    color_space_fn(material_1_color_raw, material_1->Ks);
    color_scale(material_1->Ka, 0.2000000000);
    color_scale(material_1->Kd, 0.8000000000);
    color_scale(material_1->Ks, 0.0000000000);
    rgb_to_rgb(material_1_reflective, material_1->refl);
    rgb_to_rgb(material_1_refractive, material_1->Tf);
    material_1->reflective = material_1_reflective[0] > 0.0
                             || material_1_reflective[1] > 0.0
                             || material_1_reflective[2] > 0.0;

    material_1->Tr = 0.0000000000;
    material_1->Ns = 200.0000000000;
    material_1->Ni = 1.0000000000;
    material_1->casts_shadow = true;
    material_set_pattern(material_1, map_Ka, pattern_1_Ka);
    material_set_pattern(material_1, map_Kd, pattern_1_Kd);
    material_set_pattern(material_1, map_Ks, pattern_1_Ks);
    material_set_pattern(material_1, map_Ns, pattern_1_Ns);
    material_set_pattern(material_1, map_d, pattern_1_d);
    material_set_pattern(material_1, map_bump, pattern_1_bump);
    material_set_pattern(material_1, map_disp, pattern_1_disp);
    material_set_pattern(material_1, map_refl, pattern_1_refl);

    Matrix transform_1, transform_1_tmp;
    matrix_identity(transform_1);
    matrix_rotate_y(2.3562000000, transform_1_tmp);
    transform_chain(transform_1_tmp, transform_1);
    matrix_rotate_x(0.7854000000, transform_1_tmp);
    transform_chain(transform_1_tmp, transform_1);
    matrix_translate(-2.0000000000, 2.0000000000, 0.0000000000, transform_1_tmp);
    transform_chain(transform_1_tmp, transform_1);

    Shape shape_1 = all_shapes + 1;
    cube(shape_1);
    shape_set_material(shape_1, material_1);
    shape_set_transform(shape_1, transform_1);

    /* end shape 1 */
    /* shape 2 */
    
    Matrix transform_pattern_2_Ka;
    matrix_identity(transform_pattern_2_Ka);
    Pattern pattern_2_Ka = array_of_patterns(7);
    Pattern pattern_2_Ka_right = pattern_2_Ka + 1;
    Pattern pattern_2_Ka_left = pattern_2_Ka + 2;
    Pattern pattern_2_Ka_up = pattern_2_Ka + 3;
    Pattern pattern_2_Ka_down = pattern_2_Ka + 4;
    Pattern pattern_2_Ka_front = pattern_2_Ka + 5;
    Pattern pattern_2_Ka_back = pattern_2_Ka + 6;

    Color pattern_2_Ka_right_color_0_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_2_Ka_right_color_1_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_2_Ka_right_color_2_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_2_Ka_right_color_3_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_2_Ka_right_color_4_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_2_Ka_right_color_0;
    Color pattern_2_Ka_right_color_1;
    Color pattern_2_Ka_right_color_2;
    Color pattern_2_Ka_right_color_3;
    Color pattern_2_Ka_right_color_4;
    color_space_fn(pattern_2_Ka_right_color_0_raw, pattern_2_Ka_right_color_0);
    color_space_fn(pattern_2_Ka_right_color_1_raw, pattern_2_Ka_right_color_1);
    color_space_fn(pattern_2_Ka_right_color_2_raw, pattern_2_Ka_right_color_2);
    color_space_fn(pattern_2_Ka_right_color_3_raw, pattern_2_Ka_right_color_3);
    color_space_fn(pattern_2_Ka_right_color_4_raw, pattern_2_Ka_right_color_4);
    uv_align_check_pattern(pattern_2_Ka_right_color_0, pattern_2_Ka_right_color_1, pattern_2_Ka_right_color_2, pattern_2_Ka_right_color_3, pattern_2_Ka_right_color_4, pattern_2_Ka_right);


    Color pattern_2_Ka_left_color_0_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_2_Ka_left_color_1_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_2_Ka_left_color_2_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_2_Ka_left_color_3_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_2_Ka_left_color_4_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_2_Ka_left_color_0;
    Color pattern_2_Ka_left_color_1;
    Color pattern_2_Ka_left_color_2;
    Color pattern_2_Ka_left_color_3;
    Color pattern_2_Ka_left_color_4;
    color_space_fn(pattern_2_Ka_left_color_0_raw, pattern_2_Ka_left_color_0);
    color_space_fn(pattern_2_Ka_left_color_1_raw, pattern_2_Ka_left_color_1);
    color_space_fn(pattern_2_Ka_left_color_2_raw, pattern_2_Ka_left_color_2);
    color_space_fn(pattern_2_Ka_left_color_3_raw, pattern_2_Ka_left_color_3);
    color_space_fn(pattern_2_Ka_left_color_4_raw, pattern_2_Ka_left_color_4);
    uv_align_check_pattern(pattern_2_Ka_left_color_0, pattern_2_Ka_left_color_1, pattern_2_Ka_left_color_2, pattern_2_Ka_left_color_3, pattern_2_Ka_left_color_4, pattern_2_Ka_left);


    Color pattern_2_Ka_up_color_0_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_2_Ka_up_color_1_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_2_Ka_up_color_2_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_2_Ka_up_color_3_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_2_Ka_up_color_4_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_2_Ka_up_color_0;
    Color pattern_2_Ka_up_color_1;
    Color pattern_2_Ka_up_color_2;
    Color pattern_2_Ka_up_color_3;
    Color pattern_2_Ka_up_color_4;
    color_space_fn(pattern_2_Ka_up_color_0_raw, pattern_2_Ka_up_color_0);
    color_space_fn(pattern_2_Ka_up_color_1_raw, pattern_2_Ka_up_color_1);
    color_space_fn(pattern_2_Ka_up_color_2_raw, pattern_2_Ka_up_color_2);
    color_space_fn(pattern_2_Ka_up_color_3_raw, pattern_2_Ka_up_color_3);
    color_space_fn(pattern_2_Ka_up_color_4_raw, pattern_2_Ka_up_color_4);
    uv_align_check_pattern(pattern_2_Ka_up_color_0, pattern_2_Ka_up_color_1, pattern_2_Ka_up_color_2, pattern_2_Ka_up_color_3, pattern_2_Ka_up_color_4, pattern_2_Ka_up);


    Color pattern_2_Ka_down_color_0_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_2_Ka_down_color_1_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_2_Ka_down_color_2_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_2_Ka_down_color_3_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_2_Ka_down_color_4_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_2_Ka_down_color_0;
    Color pattern_2_Ka_down_color_1;
    Color pattern_2_Ka_down_color_2;
    Color pattern_2_Ka_down_color_3;
    Color pattern_2_Ka_down_color_4;
    color_space_fn(pattern_2_Ka_down_color_0_raw, pattern_2_Ka_down_color_0);
    color_space_fn(pattern_2_Ka_down_color_1_raw, pattern_2_Ka_down_color_1);
    color_space_fn(pattern_2_Ka_down_color_2_raw, pattern_2_Ka_down_color_2);
    color_space_fn(pattern_2_Ka_down_color_3_raw, pattern_2_Ka_down_color_3);
    color_space_fn(pattern_2_Ka_down_color_4_raw, pattern_2_Ka_down_color_4);
    uv_align_check_pattern(pattern_2_Ka_down_color_0, pattern_2_Ka_down_color_1, pattern_2_Ka_down_color_2, pattern_2_Ka_down_color_3, pattern_2_Ka_down_color_4, pattern_2_Ka_down);


    Color pattern_2_Ka_front_color_0_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_2_Ka_front_color_1_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_2_Ka_front_color_2_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_2_Ka_front_color_3_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_2_Ka_front_color_4_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_2_Ka_front_color_0;
    Color pattern_2_Ka_front_color_1;
    Color pattern_2_Ka_front_color_2;
    Color pattern_2_Ka_front_color_3;
    Color pattern_2_Ka_front_color_4;
    color_space_fn(pattern_2_Ka_front_color_0_raw, pattern_2_Ka_front_color_0);
    color_space_fn(pattern_2_Ka_front_color_1_raw, pattern_2_Ka_front_color_1);
    color_space_fn(pattern_2_Ka_front_color_2_raw, pattern_2_Ka_front_color_2);
    color_space_fn(pattern_2_Ka_front_color_3_raw, pattern_2_Ka_front_color_3);
    color_space_fn(pattern_2_Ka_front_color_4_raw, pattern_2_Ka_front_color_4);
    uv_align_check_pattern(pattern_2_Ka_front_color_0, pattern_2_Ka_front_color_1, pattern_2_Ka_front_color_2, pattern_2_Ka_front_color_3, pattern_2_Ka_front_color_4, pattern_2_Ka_front);


    Color pattern_2_Ka_back_color_0_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_2_Ka_back_color_1_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_2_Ka_back_color_2_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_2_Ka_back_color_3_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_2_Ka_back_color_4_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_2_Ka_back_color_0;
    Color pattern_2_Ka_back_color_1;
    Color pattern_2_Ka_back_color_2;
    Color pattern_2_Ka_back_color_3;
    Color pattern_2_Ka_back_color_4;
    color_space_fn(pattern_2_Ka_back_color_0_raw, pattern_2_Ka_back_color_0);
    color_space_fn(pattern_2_Ka_back_color_1_raw, pattern_2_Ka_back_color_1);
    color_space_fn(pattern_2_Ka_back_color_2_raw, pattern_2_Ka_back_color_2);
    color_space_fn(pattern_2_Ka_back_color_3_raw, pattern_2_Ka_back_color_3);
    color_space_fn(pattern_2_Ka_back_color_4_raw, pattern_2_Ka_back_color_4);
    uv_align_check_pattern(pattern_2_Ka_back_color_0, pattern_2_Ka_back_color_1, pattern_2_Ka_back_color_2, pattern_2_Ka_back_color_3, pattern_2_Ka_back_color_4, pattern_2_Ka_back);



    texture_map_pattern(pattern_2_Ka_right, CUBE_UV_MAP, pattern_2_Ka);
    pattern_set_transform(pattern_2_Ka, transform_pattern_2_Ka);
Matrix transform_pattern_2_Kd;
    matrix_identity(transform_pattern_2_Kd);
    Pattern pattern_2_Kd = array_of_patterns(7);
    Pattern pattern_2_Kd_right = pattern_2_Kd + 1;
    Pattern pattern_2_Kd_left = pattern_2_Kd + 2;
    Pattern pattern_2_Kd_up = pattern_2_Kd + 3;
    Pattern pattern_2_Kd_down = pattern_2_Kd + 4;
    Pattern pattern_2_Kd_front = pattern_2_Kd + 5;
    Pattern pattern_2_Kd_back = pattern_2_Kd + 6;

    Color pattern_2_Kd_right_color_0_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_2_Kd_right_color_1_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_2_Kd_right_color_2_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_2_Kd_right_color_3_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_2_Kd_right_color_4_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_2_Kd_right_color_0;
    Color pattern_2_Kd_right_color_1;
    Color pattern_2_Kd_right_color_2;
    Color pattern_2_Kd_right_color_3;
    Color pattern_2_Kd_right_color_4;
    color_space_fn(pattern_2_Kd_right_color_0_raw, pattern_2_Kd_right_color_0);
    color_space_fn(pattern_2_Kd_right_color_1_raw, pattern_2_Kd_right_color_1);
    color_space_fn(pattern_2_Kd_right_color_2_raw, pattern_2_Kd_right_color_2);
    color_space_fn(pattern_2_Kd_right_color_3_raw, pattern_2_Kd_right_color_3);
    color_space_fn(pattern_2_Kd_right_color_4_raw, pattern_2_Kd_right_color_4);
    uv_align_check_pattern(pattern_2_Kd_right_color_0, pattern_2_Kd_right_color_1, pattern_2_Kd_right_color_2, pattern_2_Kd_right_color_3, pattern_2_Kd_right_color_4, pattern_2_Kd_right);


    Color pattern_2_Kd_left_color_0_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_2_Kd_left_color_1_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_2_Kd_left_color_2_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_2_Kd_left_color_3_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_2_Kd_left_color_4_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_2_Kd_left_color_0;
    Color pattern_2_Kd_left_color_1;
    Color pattern_2_Kd_left_color_2;
    Color pattern_2_Kd_left_color_3;
    Color pattern_2_Kd_left_color_4;
    color_space_fn(pattern_2_Kd_left_color_0_raw, pattern_2_Kd_left_color_0);
    color_space_fn(pattern_2_Kd_left_color_1_raw, pattern_2_Kd_left_color_1);
    color_space_fn(pattern_2_Kd_left_color_2_raw, pattern_2_Kd_left_color_2);
    color_space_fn(pattern_2_Kd_left_color_3_raw, pattern_2_Kd_left_color_3);
    color_space_fn(pattern_2_Kd_left_color_4_raw, pattern_2_Kd_left_color_4);
    uv_align_check_pattern(pattern_2_Kd_left_color_0, pattern_2_Kd_left_color_1, pattern_2_Kd_left_color_2, pattern_2_Kd_left_color_3, pattern_2_Kd_left_color_4, pattern_2_Kd_left);


    Color pattern_2_Kd_up_color_0_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_2_Kd_up_color_1_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_2_Kd_up_color_2_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_2_Kd_up_color_3_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_2_Kd_up_color_4_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_2_Kd_up_color_0;
    Color pattern_2_Kd_up_color_1;
    Color pattern_2_Kd_up_color_2;
    Color pattern_2_Kd_up_color_3;
    Color pattern_2_Kd_up_color_4;
    color_space_fn(pattern_2_Kd_up_color_0_raw, pattern_2_Kd_up_color_0);
    color_space_fn(pattern_2_Kd_up_color_1_raw, pattern_2_Kd_up_color_1);
    color_space_fn(pattern_2_Kd_up_color_2_raw, pattern_2_Kd_up_color_2);
    color_space_fn(pattern_2_Kd_up_color_3_raw, pattern_2_Kd_up_color_3);
    color_space_fn(pattern_2_Kd_up_color_4_raw, pattern_2_Kd_up_color_4);
    uv_align_check_pattern(pattern_2_Kd_up_color_0, pattern_2_Kd_up_color_1, pattern_2_Kd_up_color_2, pattern_2_Kd_up_color_3, pattern_2_Kd_up_color_4, pattern_2_Kd_up);


    Color pattern_2_Kd_down_color_0_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_2_Kd_down_color_1_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_2_Kd_down_color_2_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_2_Kd_down_color_3_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_2_Kd_down_color_4_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_2_Kd_down_color_0;
    Color pattern_2_Kd_down_color_1;
    Color pattern_2_Kd_down_color_2;
    Color pattern_2_Kd_down_color_3;
    Color pattern_2_Kd_down_color_4;
    color_space_fn(pattern_2_Kd_down_color_0_raw, pattern_2_Kd_down_color_0);
    color_space_fn(pattern_2_Kd_down_color_1_raw, pattern_2_Kd_down_color_1);
    color_space_fn(pattern_2_Kd_down_color_2_raw, pattern_2_Kd_down_color_2);
    color_space_fn(pattern_2_Kd_down_color_3_raw, pattern_2_Kd_down_color_3);
    color_space_fn(pattern_2_Kd_down_color_4_raw, pattern_2_Kd_down_color_4);
    uv_align_check_pattern(pattern_2_Kd_down_color_0, pattern_2_Kd_down_color_1, pattern_2_Kd_down_color_2, pattern_2_Kd_down_color_3, pattern_2_Kd_down_color_4, pattern_2_Kd_down);


    Color pattern_2_Kd_front_color_0_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_2_Kd_front_color_1_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_2_Kd_front_color_2_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_2_Kd_front_color_3_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_2_Kd_front_color_4_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_2_Kd_front_color_0;
    Color pattern_2_Kd_front_color_1;
    Color pattern_2_Kd_front_color_2;
    Color pattern_2_Kd_front_color_3;
    Color pattern_2_Kd_front_color_4;
    color_space_fn(pattern_2_Kd_front_color_0_raw, pattern_2_Kd_front_color_0);
    color_space_fn(pattern_2_Kd_front_color_1_raw, pattern_2_Kd_front_color_1);
    color_space_fn(pattern_2_Kd_front_color_2_raw, pattern_2_Kd_front_color_2);
    color_space_fn(pattern_2_Kd_front_color_3_raw, pattern_2_Kd_front_color_3);
    color_space_fn(pattern_2_Kd_front_color_4_raw, pattern_2_Kd_front_color_4);
    uv_align_check_pattern(pattern_2_Kd_front_color_0, pattern_2_Kd_front_color_1, pattern_2_Kd_front_color_2, pattern_2_Kd_front_color_3, pattern_2_Kd_front_color_4, pattern_2_Kd_front);


    Color pattern_2_Kd_back_color_0_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_2_Kd_back_color_1_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_2_Kd_back_color_2_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_2_Kd_back_color_3_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_2_Kd_back_color_4_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_2_Kd_back_color_0;
    Color pattern_2_Kd_back_color_1;
    Color pattern_2_Kd_back_color_2;
    Color pattern_2_Kd_back_color_3;
    Color pattern_2_Kd_back_color_4;
    color_space_fn(pattern_2_Kd_back_color_0_raw, pattern_2_Kd_back_color_0);
    color_space_fn(pattern_2_Kd_back_color_1_raw, pattern_2_Kd_back_color_1);
    color_space_fn(pattern_2_Kd_back_color_2_raw, pattern_2_Kd_back_color_2);
    color_space_fn(pattern_2_Kd_back_color_3_raw, pattern_2_Kd_back_color_3);
    color_space_fn(pattern_2_Kd_back_color_4_raw, pattern_2_Kd_back_color_4);
    uv_align_check_pattern(pattern_2_Kd_back_color_0, pattern_2_Kd_back_color_1, pattern_2_Kd_back_color_2, pattern_2_Kd_back_color_3, pattern_2_Kd_back_color_4, pattern_2_Kd_back);



    texture_map_pattern(pattern_2_Kd_right, CUBE_UV_MAP, pattern_2_Kd);
    pattern_set_transform(pattern_2_Kd, transform_pattern_2_Kd);
    Pattern pattern_2_Ks = NULL;
    Pattern pattern_2_Ns = NULL;
    Pattern pattern_2_bump = NULL;
    Pattern pattern_2_disp = NULL;
    Pattern pattern_2_refl = NULL;
    Pattern pattern_2_d = NULL;
    Color material_2_color_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color material_2_reflective = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_2_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_2 = material_alloc();
    color_space_fn(material_2_color_raw, material_2->Ka);
    color_space_fn(material_2_color_raw, material_2->Kd);
    color_space_fn(material_2_color_raw, material_2->Ks);
    color_scale(material_2->Ka, 0.2000000000);
    color_scale(material_2->Kd, 0.8000000000);
    color_scale(material_2->Ks, 0.0000000000);
    rgb_to_rgb(material_2_reflective, material_2->refl);
    rgb_to_rgb(material_2_refractive, material_2->Tf);
    material_2->reflective = material_2_reflective[0] > 0.0
                             || material_2_reflective[1] > 0.0
                             || material_2_reflective[2] > 0.0;

    material_2->Tr = 0.0000000000;
    material_2->Ns = 200.0000000000;
    material_2->Ni = 1.0000000000;
    material_2->casts_shadow = true;
    material_set_pattern(material_2, map_Ka, pattern_2_Ka);
    material_set_pattern(material_2, map_Kd, pattern_2_Kd);
    material_set_pattern(material_2, map_Ks, pattern_2_Ks);
    material_set_pattern(material_2, map_Ns, pattern_2_Ns);
    material_set_pattern(material_2, map_d, pattern_2_d);
    material_set_pattern(material_2, map_bump, pattern_2_bump);
    material_set_pattern(material_2, map_disp, pattern_2_disp);
    material_set_pattern(material_2, map_refl, pattern_2_refl);

    Matrix transform_2, transform_2_tmp;
    matrix_identity(transform_2);
    matrix_rotate_y(3.9270000000, transform_2_tmp);
    transform_chain(transform_2_tmp, transform_2);
    matrix_rotate_x(0.7854000000, transform_2_tmp);
    transform_chain(transform_2_tmp, transform_2);
    matrix_translate(2.0000000000, 2.0000000000, 0.0000000000, transform_2_tmp);
    transform_chain(transform_2_tmp, transform_2);

    Shape shape_2 = all_shapes + 2;
    cube(shape_2);
    shape_set_material(shape_2, material_2);
    shape_set_transform(shape_2, transform_2);

    /* end shape 2 */
    /* shape 3 */
    
    Matrix transform_pattern_3_Ka;
    matrix_identity(transform_pattern_3_Ka);
    Pattern pattern_3_Ka = array_of_patterns(7);
    Pattern pattern_3_Ka_right = pattern_3_Ka + 1;
    Pattern pattern_3_Ka_left = pattern_3_Ka + 2;
    Pattern pattern_3_Ka_up = pattern_3_Ka + 3;
    Pattern pattern_3_Ka_down = pattern_3_Ka + 4;
    Pattern pattern_3_Ka_front = pattern_3_Ka + 5;
    Pattern pattern_3_Ka_back = pattern_3_Ka + 6;

    Color pattern_3_Ka_right_color_0_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_3_Ka_right_color_1_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_3_Ka_right_color_2_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_3_Ka_right_color_3_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_3_Ka_right_color_4_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_3_Ka_right_color_0;
    Color pattern_3_Ka_right_color_1;
    Color pattern_3_Ka_right_color_2;
    Color pattern_3_Ka_right_color_3;
    Color pattern_3_Ka_right_color_4;
    color_space_fn(pattern_3_Ka_right_color_0_raw, pattern_3_Ka_right_color_0);
    color_space_fn(pattern_3_Ka_right_color_1_raw, pattern_3_Ka_right_color_1);
    color_space_fn(pattern_3_Ka_right_color_2_raw, pattern_3_Ka_right_color_2);
    color_space_fn(pattern_3_Ka_right_color_3_raw, pattern_3_Ka_right_color_3);
    color_space_fn(pattern_3_Ka_right_color_4_raw, pattern_3_Ka_right_color_4);
    uv_align_check_pattern(pattern_3_Ka_right_color_0, pattern_3_Ka_right_color_1, pattern_3_Ka_right_color_2, pattern_3_Ka_right_color_3, pattern_3_Ka_right_color_4, pattern_3_Ka_right);


    Color pattern_3_Ka_left_color_0_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_3_Ka_left_color_1_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_3_Ka_left_color_2_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_3_Ka_left_color_3_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_3_Ka_left_color_4_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_3_Ka_left_color_0;
    Color pattern_3_Ka_left_color_1;
    Color pattern_3_Ka_left_color_2;
    Color pattern_3_Ka_left_color_3;
    Color pattern_3_Ka_left_color_4;
    color_space_fn(pattern_3_Ka_left_color_0_raw, pattern_3_Ka_left_color_0);
    color_space_fn(pattern_3_Ka_left_color_1_raw, pattern_3_Ka_left_color_1);
    color_space_fn(pattern_3_Ka_left_color_2_raw, pattern_3_Ka_left_color_2);
    color_space_fn(pattern_3_Ka_left_color_3_raw, pattern_3_Ka_left_color_3);
    color_space_fn(pattern_3_Ka_left_color_4_raw, pattern_3_Ka_left_color_4);
    uv_align_check_pattern(pattern_3_Ka_left_color_0, pattern_3_Ka_left_color_1, pattern_3_Ka_left_color_2, pattern_3_Ka_left_color_3, pattern_3_Ka_left_color_4, pattern_3_Ka_left);


    Color pattern_3_Ka_up_color_0_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_3_Ka_up_color_1_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_3_Ka_up_color_2_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_3_Ka_up_color_3_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_3_Ka_up_color_4_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_3_Ka_up_color_0;
    Color pattern_3_Ka_up_color_1;
    Color pattern_3_Ka_up_color_2;
    Color pattern_3_Ka_up_color_3;
    Color pattern_3_Ka_up_color_4;
    color_space_fn(pattern_3_Ka_up_color_0_raw, pattern_3_Ka_up_color_0);
    color_space_fn(pattern_3_Ka_up_color_1_raw, pattern_3_Ka_up_color_1);
    color_space_fn(pattern_3_Ka_up_color_2_raw, pattern_3_Ka_up_color_2);
    color_space_fn(pattern_3_Ka_up_color_3_raw, pattern_3_Ka_up_color_3);
    color_space_fn(pattern_3_Ka_up_color_4_raw, pattern_3_Ka_up_color_4);
    uv_align_check_pattern(pattern_3_Ka_up_color_0, pattern_3_Ka_up_color_1, pattern_3_Ka_up_color_2, pattern_3_Ka_up_color_3, pattern_3_Ka_up_color_4, pattern_3_Ka_up);


    Color pattern_3_Ka_down_color_0_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_3_Ka_down_color_1_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_3_Ka_down_color_2_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_3_Ka_down_color_3_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_3_Ka_down_color_4_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_3_Ka_down_color_0;
    Color pattern_3_Ka_down_color_1;
    Color pattern_3_Ka_down_color_2;
    Color pattern_3_Ka_down_color_3;
    Color pattern_3_Ka_down_color_4;
    color_space_fn(pattern_3_Ka_down_color_0_raw, pattern_3_Ka_down_color_0);
    color_space_fn(pattern_3_Ka_down_color_1_raw, pattern_3_Ka_down_color_1);
    color_space_fn(pattern_3_Ka_down_color_2_raw, pattern_3_Ka_down_color_2);
    color_space_fn(pattern_3_Ka_down_color_3_raw, pattern_3_Ka_down_color_3);
    color_space_fn(pattern_3_Ka_down_color_4_raw, pattern_3_Ka_down_color_4);
    uv_align_check_pattern(pattern_3_Ka_down_color_0, pattern_3_Ka_down_color_1, pattern_3_Ka_down_color_2, pattern_3_Ka_down_color_3, pattern_3_Ka_down_color_4, pattern_3_Ka_down);


    Color pattern_3_Ka_front_color_0_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_3_Ka_front_color_1_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_3_Ka_front_color_2_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_3_Ka_front_color_3_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_3_Ka_front_color_4_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_3_Ka_front_color_0;
    Color pattern_3_Ka_front_color_1;
    Color pattern_3_Ka_front_color_2;
    Color pattern_3_Ka_front_color_3;
    Color pattern_3_Ka_front_color_4;
    color_space_fn(pattern_3_Ka_front_color_0_raw, pattern_3_Ka_front_color_0);
    color_space_fn(pattern_3_Ka_front_color_1_raw, pattern_3_Ka_front_color_1);
    color_space_fn(pattern_3_Ka_front_color_2_raw, pattern_3_Ka_front_color_2);
    color_space_fn(pattern_3_Ka_front_color_3_raw, pattern_3_Ka_front_color_3);
    color_space_fn(pattern_3_Ka_front_color_4_raw, pattern_3_Ka_front_color_4);
    uv_align_check_pattern(pattern_3_Ka_front_color_0, pattern_3_Ka_front_color_1, pattern_3_Ka_front_color_2, pattern_3_Ka_front_color_3, pattern_3_Ka_front_color_4, pattern_3_Ka_front);


    Color pattern_3_Ka_back_color_0_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_3_Ka_back_color_1_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_3_Ka_back_color_2_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_3_Ka_back_color_3_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_3_Ka_back_color_4_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_3_Ka_back_color_0;
    Color pattern_3_Ka_back_color_1;
    Color pattern_3_Ka_back_color_2;
    Color pattern_3_Ka_back_color_3;
    Color pattern_3_Ka_back_color_4;
    color_space_fn(pattern_3_Ka_back_color_0_raw, pattern_3_Ka_back_color_0);
    color_space_fn(pattern_3_Ka_back_color_1_raw, pattern_3_Ka_back_color_1);
    color_space_fn(pattern_3_Ka_back_color_2_raw, pattern_3_Ka_back_color_2);
    color_space_fn(pattern_3_Ka_back_color_3_raw, pattern_3_Ka_back_color_3);
    color_space_fn(pattern_3_Ka_back_color_4_raw, pattern_3_Ka_back_color_4);
    uv_align_check_pattern(pattern_3_Ka_back_color_0, pattern_3_Ka_back_color_1, pattern_3_Ka_back_color_2, pattern_3_Ka_back_color_3, pattern_3_Ka_back_color_4, pattern_3_Ka_back);



    texture_map_pattern(pattern_3_Ka_right, CUBE_UV_MAP, pattern_3_Ka);
    pattern_set_transform(pattern_3_Ka, transform_pattern_3_Ka);
Matrix transform_pattern_3_Kd;
    matrix_identity(transform_pattern_3_Kd);
    Pattern pattern_3_Kd = array_of_patterns(7);
    Pattern pattern_3_Kd_right = pattern_3_Kd + 1;
    Pattern pattern_3_Kd_left = pattern_3_Kd + 2;
    Pattern pattern_3_Kd_up = pattern_3_Kd + 3;
    Pattern pattern_3_Kd_down = pattern_3_Kd + 4;
    Pattern pattern_3_Kd_front = pattern_3_Kd + 5;
    Pattern pattern_3_Kd_back = pattern_3_Kd + 6;

    Color pattern_3_Kd_right_color_0_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_3_Kd_right_color_1_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_3_Kd_right_color_2_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_3_Kd_right_color_3_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_3_Kd_right_color_4_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_3_Kd_right_color_0;
    Color pattern_3_Kd_right_color_1;
    Color pattern_3_Kd_right_color_2;
    Color pattern_3_Kd_right_color_3;
    Color pattern_3_Kd_right_color_4;
    color_space_fn(pattern_3_Kd_right_color_0_raw, pattern_3_Kd_right_color_0);
    color_space_fn(pattern_3_Kd_right_color_1_raw, pattern_3_Kd_right_color_1);
    color_space_fn(pattern_3_Kd_right_color_2_raw, pattern_3_Kd_right_color_2);
    color_space_fn(pattern_3_Kd_right_color_3_raw, pattern_3_Kd_right_color_3);
    color_space_fn(pattern_3_Kd_right_color_4_raw, pattern_3_Kd_right_color_4);
    uv_align_check_pattern(pattern_3_Kd_right_color_0, pattern_3_Kd_right_color_1, pattern_3_Kd_right_color_2, pattern_3_Kd_right_color_3, pattern_3_Kd_right_color_4, pattern_3_Kd_right);


    Color pattern_3_Kd_left_color_0_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_3_Kd_left_color_1_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_3_Kd_left_color_2_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_3_Kd_left_color_3_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_3_Kd_left_color_4_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_3_Kd_left_color_0;
    Color pattern_3_Kd_left_color_1;
    Color pattern_3_Kd_left_color_2;
    Color pattern_3_Kd_left_color_3;
    Color pattern_3_Kd_left_color_4;
    color_space_fn(pattern_3_Kd_left_color_0_raw, pattern_3_Kd_left_color_0);
    color_space_fn(pattern_3_Kd_left_color_1_raw, pattern_3_Kd_left_color_1);
    color_space_fn(pattern_3_Kd_left_color_2_raw, pattern_3_Kd_left_color_2);
    color_space_fn(pattern_3_Kd_left_color_3_raw, pattern_3_Kd_left_color_3);
    color_space_fn(pattern_3_Kd_left_color_4_raw, pattern_3_Kd_left_color_4);
    uv_align_check_pattern(pattern_3_Kd_left_color_0, pattern_3_Kd_left_color_1, pattern_3_Kd_left_color_2, pattern_3_Kd_left_color_3, pattern_3_Kd_left_color_4, pattern_3_Kd_left);


    Color pattern_3_Kd_up_color_0_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_3_Kd_up_color_1_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_3_Kd_up_color_2_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_3_Kd_up_color_3_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_3_Kd_up_color_4_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_3_Kd_up_color_0;
    Color pattern_3_Kd_up_color_1;
    Color pattern_3_Kd_up_color_2;
    Color pattern_3_Kd_up_color_3;
    Color pattern_3_Kd_up_color_4;
    color_space_fn(pattern_3_Kd_up_color_0_raw, pattern_3_Kd_up_color_0);
    color_space_fn(pattern_3_Kd_up_color_1_raw, pattern_3_Kd_up_color_1);
    color_space_fn(pattern_3_Kd_up_color_2_raw, pattern_3_Kd_up_color_2);
    color_space_fn(pattern_3_Kd_up_color_3_raw, pattern_3_Kd_up_color_3);
    color_space_fn(pattern_3_Kd_up_color_4_raw, pattern_3_Kd_up_color_4);
    uv_align_check_pattern(pattern_3_Kd_up_color_0, pattern_3_Kd_up_color_1, pattern_3_Kd_up_color_2, pattern_3_Kd_up_color_3, pattern_3_Kd_up_color_4, pattern_3_Kd_up);


    Color pattern_3_Kd_down_color_0_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_3_Kd_down_color_1_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_3_Kd_down_color_2_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_3_Kd_down_color_3_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_3_Kd_down_color_4_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_3_Kd_down_color_0;
    Color pattern_3_Kd_down_color_1;
    Color pattern_3_Kd_down_color_2;
    Color pattern_3_Kd_down_color_3;
    Color pattern_3_Kd_down_color_4;
    color_space_fn(pattern_3_Kd_down_color_0_raw, pattern_3_Kd_down_color_0);
    color_space_fn(pattern_3_Kd_down_color_1_raw, pattern_3_Kd_down_color_1);
    color_space_fn(pattern_3_Kd_down_color_2_raw, pattern_3_Kd_down_color_2);
    color_space_fn(pattern_3_Kd_down_color_3_raw, pattern_3_Kd_down_color_3);
    color_space_fn(pattern_3_Kd_down_color_4_raw, pattern_3_Kd_down_color_4);
    uv_align_check_pattern(pattern_3_Kd_down_color_0, pattern_3_Kd_down_color_1, pattern_3_Kd_down_color_2, pattern_3_Kd_down_color_3, pattern_3_Kd_down_color_4, pattern_3_Kd_down);


    Color pattern_3_Kd_front_color_0_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_3_Kd_front_color_1_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_3_Kd_front_color_2_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_3_Kd_front_color_3_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_3_Kd_front_color_4_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_3_Kd_front_color_0;
    Color pattern_3_Kd_front_color_1;
    Color pattern_3_Kd_front_color_2;
    Color pattern_3_Kd_front_color_3;
    Color pattern_3_Kd_front_color_4;
    color_space_fn(pattern_3_Kd_front_color_0_raw, pattern_3_Kd_front_color_0);
    color_space_fn(pattern_3_Kd_front_color_1_raw, pattern_3_Kd_front_color_1);
    color_space_fn(pattern_3_Kd_front_color_2_raw, pattern_3_Kd_front_color_2);
    color_space_fn(pattern_3_Kd_front_color_3_raw, pattern_3_Kd_front_color_3);
    color_space_fn(pattern_3_Kd_front_color_4_raw, pattern_3_Kd_front_color_4);
    uv_align_check_pattern(pattern_3_Kd_front_color_0, pattern_3_Kd_front_color_1, pattern_3_Kd_front_color_2, pattern_3_Kd_front_color_3, pattern_3_Kd_front_color_4, pattern_3_Kd_front);


    Color pattern_3_Kd_back_color_0_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_3_Kd_back_color_1_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_3_Kd_back_color_2_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_3_Kd_back_color_3_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_3_Kd_back_color_4_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_3_Kd_back_color_0;
    Color pattern_3_Kd_back_color_1;
    Color pattern_3_Kd_back_color_2;
    Color pattern_3_Kd_back_color_3;
    Color pattern_3_Kd_back_color_4;
    color_space_fn(pattern_3_Kd_back_color_0_raw, pattern_3_Kd_back_color_0);
    color_space_fn(pattern_3_Kd_back_color_1_raw, pattern_3_Kd_back_color_1);
    color_space_fn(pattern_3_Kd_back_color_2_raw, pattern_3_Kd_back_color_2);
    color_space_fn(pattern_3_Kd_back_color_3_raw, pattern_3_Kd_back_color_3);
    color_space_fn(pattern_3_Kd_back_color_4_raw, pattern_3_Kd_back_color_4);
    uv_align_check_pattern(pattern_3_Kd_back_color_0, pattern_3_Kd_back_color_1, pattern_3_Kd_back_color_2, pattern_3_Kd_back_color_3, pattern_3_Kd_back_color_4, pattern_3_Kd_back);



    texture_map_pattern(pattern_3_Kd_right, CUBE_UV_MAP, pattern_3_Kd);
    pattern_set_transform(pattern_3_Kd, transform_pattern_3_Kd);
    Pattern pattern_3_Ks = NULL;
    Pattern pattern_3_Ns = NULL;
    Pattern pattern_3_bump = NULL;
    Pattern pattern_3_disp = NULL;
    Pattern pattern_3_refl = NULL;
    Pattern pattern_3_d = NULL;
    Color material_3_color_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color material_3_reflective = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_3_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_3 = material_alloc();
    color_space_fn(material_3_color_raw, material_3->Ka);
    color_space_fn(material_3_color_raw, material_3->Kd);
    color_space_fn(material_3_color_raw, material_3->Ks);
    color_scale(material_3->Ka, 0.2000000000);
    color_scale(material_3->Kd, 0.8000000000);
    color_scale(material_3->Ks, 0.0000000000);
    rgb_to_rgb(material_3_reflective, material_3->refl);
    rgb_to_rgb(material_3_refractive, material_3->Tf);
    material_3->reflective = material_3_reflective[0] > 0.0
                             || material_3_reflective[1] > 0.0
                             || material_3_reflective[2] > 0.0;

    material_3->Tr = 0.0000000000;
    material_3->Ns = 200.0000000000;
    material_3->Ni = 1.0000000000;
    material_3->casts_shadow = true;
    material_set_pattern(material_3, map_Ka, pattern_3_Ka);
    material_set_pattern(material_3, map_Kd, pattern_3_Kd);
    material_set_pattern(material_3, map_Ks, pattern_3_Ks);
    material_set_pattern(material_3, map_Ns, pattern_3_Ns);
    material_set_pattern(material_3, map_d, pattern_3_d);
    material_set_pattern(material_3, map_bump, pattern_3_bump);
    material_set_pattern(material_3, map_disp, pattern_3_disp);
    material_set_pattern(material_3, map_refl, pattern_3_refl);

    Matrix transform_3, transform_3_tmp;
    matrix_identity(transform_3);
    matrix_rotate_y(5.4978000000, transform_3_tmp);
    transform_chain(transform_3_tmp, transform_3);
    matrix_rotate_x(0.7854000000, transform_3_tmp);
    transform_chain(transform_3_tmp, transform_3);
    matrix_translate(6.0000000000, 2.0000000000, 0.0000000000, transform_3_tmp);
    transform_chain(transform_3_tmp, transform_3);

    Shape shape_3 = all_shapes + 3;
    cube(shape_3);
    shape_set_material(shape_3, material_3);
    shape_set_transform(shape_3, transform_3);

    /* end shape 3 */
    /* shape 4 */
    
    Matrix transform_pattern_4_Ka;
    matrix_identity(transform_pattern_4_Ka);
    Pattern pattern_4_Ka = array_of_patterns(7);
    Pattern pattern_4_Ka_right = pattern_4_Ka + 1;
    Pattern pattern_4_Ka_left = pattern_4_Ka + 2;
    Pattern pattern_4_Ka_up = pattern_4_Ka + 3;
    Pattern pattern_4_Ka_down = pattern_4_Ka + 4;
    Pattern pattern_4_Ka_front = pattern_4_Ka + 5;
    Pattern pattern_4_Ka_back = pattern_4_Ka + 6;

    Color pattern_4_Ka_right_color_0_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_4_Ka_right_color_1_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_4_Ka_right_color_2_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_4_Ka_right_color_3_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_4_Ka_right_color_4_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_4_Ka_right_color_0;
    Color pattern_4_Ka_right_color_1;
    Color pattern_4_Ka_right_color_2;
    Color pattern_4_Ka_right_color_3;
    Color pattern_4_Ka_right_color_4;
    color_space_fn(pattern_4_Ka_right_color_0_raw, pattern_4_Ka_right_color_0);
    color_space_fn(pattern_4_Ka_right_color_1_raw, pattern_4_Ka_right_color_1);
    color_space_fn(pattern_4_Ka_right_color_2_raw, pattern_4_Ka_right_color_2);
    color_space_fn(pattern_4_Ka_right_color_3_raw, pattern_4_Ka_right_color_3);
    color_space_fn(pattern_4_Ka_right_color_4_raw, pattern_4_Ka_right_color_4);
    uv_align_check_pattern(pattern_4_Ka_right_color_0, pattern_4_Ka_right_color_1, pattern_4_Ka_right_color_2, pattern_4_Ka_right_color_3, pattern_4_Ka_right_color_4, pattern_4_Ka_right);


    Color pattern_4_Ka_left_color_0_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_4_Ka_left_color_1_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_4_Ka_left_color_2_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_4_Ka_left_color_3_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_4_Ka_left_color_4_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_4_Ka_left_color_0;
    Color pattern_4_Ka_left_color_1;
    Color pattern_4_Ka_left_color_2;
    Color pattern_4_Ka_left_color_3;
    Color pattern_4_Ka_left_color_4;
    color_space_fn(pattern_4_Ka_left_color_0_raw, pattern_4_Ka_left_color_0);
    color_space_fn(pattern_4_Ka_left_color_1_raw, pattern_4_Ka_left_color_1);
    color_space_fn(pattern_4_Ka_left_color_2_raw, pattern_4_Ka_left_color_2);
    color_space_fn(pattern_4_Ka_left_color_3_raw, pattern_4_Ka_left_color_3);
    color_space_fn(pattern_4_Ka_left_color_4_raw, pattern_4_Ka_left_color_4);
    uv_align_check_pattern(pattern_4_Ka_left_color_0, pattern_4_Ka_left_color_1, pattern_4_Ka_left_color_2, pattern_4_Ka_left_color_3, pattern_4_Ka_left_color_4, pattern_4_Ka_left);


    Color pattern_4_Ka_up_color_0_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_4_Ka_up_color_1_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_4_Ka_up_color_2_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_4_Ka_up_color_3_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_4_Ka_up_color_4_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_4_Ka_up_color_0;
    Color pattern_4_Ka_up_color_1;
    Color pattern_4_Ka_up_color_2;
    Color pattern_4_Ka_up_color_3;
    Color pattern_4_Ka_up_color_4;
    color_space_fn(pattern_4_Ka_up_color_0_raw, pattern_4_Ka_up_color_0);
    color_space_fn(pattern_4_Ka_up_color_1_raw, pattern_4_Ka_up_color_1);
    color_space_fn(pattern_4_Ka_up_color_2_raw, pattern_4_Ka_up_color_2);
    color_space_fn(pattern_4_Ka_up_color_3_raw, pattern_4_Ka_up_color_3);
    color_space_fn(pattern_4_Ka_up_color_4_raw, pattern_4_Ka_up_color_4);
    uv_align_check_pattern(pattern_4_Ka_up_color_0, pattern_4_Ka_up_color_1, pattern_4_Ka_up_color_2, pattern_4_Ka_up_color_3, pattern_4_Ka_up_color_4, pattern_4_Ka_up);


    Color pattern_4_Ka_down_color_0_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_4_Ka_down_color_1_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_4_Ka_down_color_2_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_4_Ka_down_color_3_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_4_Ka_down_color_4_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_4_Ka_down_color_0;
    Color pattern_4_Ka_down_color_1;
    Color pattern_4_Ka_down_color_2;
    Color pattern_4_Ka_down_color_3;
    Color pattern_4_Ka_down_color_4;
    color_space_fn(pattern_4_Ka_down_color_0_raw, pattern_4_Ka_down_color_0);
    color_space_fn(pattern_4_Ka_down_color_1_raw, pattern_4_Ka_down_color_1);
    color_space_fn(pattern_4_Ka_down_color_2_raw, pattern_4_Ka_down_color_2);
    color_space_fn(pattern_4_Ka_down_color_3_raw, pattern_4_Ka_down_color_3);
    color_space_fn(pattern_4_Ka_down_color_4_raw, pattern_4_Ka_down_color_4);
    uv_align_check_pattern(pattern_4_Ka_down_color_0, pattern_4_Ka_down_color_1, pattern_4_Ka_down_color_2, pattern_4_Ka_down_color_3, pattern_4_Ka_down_color_4, pattern_4_Ka_down);


    Color pattern_4_Ka_front_color_0_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_4_Ka_front_color_1_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_4_Ka_front_color_2_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_4_Ka_front_color_3_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_4_Ka_front_color_4_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_4_Ka_front_color_0;
    Color pattern_4_Ka_front_color_1;
    Color pattern_4_Ka_front_color_2;
    Color pattern_4_Ka_front_color_3;
    Color pattern_4_Ka_front_color_4;
    color_space_fn(pattern_4_Ka_front_color_0_raw, pattern_4_Ka_front_color_0);
    color_space_fn(pattern_4_Ka_front_color_1_raw, pattern_4_Ka_front_color_1);
    color_space_fn(pattern_4_Ka_front_color_2_raw, pattern_4_Ka_front_color_2);
    color_space_fn(pattern_4_Ka_front_color_3_raw, pattern_4_Ka_front_color_3);
    color_space_fn(pattern_4_Ka_front_color_4_raw, pattern_4_Ka_front_color_4);
    uv_align_check_pattern(pattern_4_Ka_front_color_0, pattern_4_Ka_front_color_1, pattern_4_Ka_front_color_2, pattern_4_Ka_front_color_3, pattern_4_Ka_front_color_4, pattern_4_Ka_front);


    Color pattern_4_Ka_back_color_0_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_4_Ka_back_color_1_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_4_Ka_back_color_2_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_4_Ka_back_color_3_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_4_Ka_back_color_4_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_4_Ka_back_color_0;
    Color pattern_4_Ka_back_color_1;
    Color pattern_4_Ka_back_color_2;
    Color pattern_4_Ka_back_color_3;
    Color pattern_4_Ka_back_color_4;
    color_space_fn(pattern_4_Ka_back_color_0_raw, pattern_4_Ka_back_color_0);
    color_space_fn(pattern_4_Ka_back_color_1_raw, pattern_4_Ka_back_color_1);
    color_space_fn(pattern_4_Ka_back_color_2_raw, pattern_4_Ka_back_color_2);
    color_space_fn(pattern_4_Ka_back_color_3_raw, pattern_4_Ka_back_color_3);
    color_space_fn(pattern_4_Ka_back_color_4_raw, pattern_4_Ka_back_color_4);
    uv_align_check_pattern(pattern_4_Ka_back_color_0, pattern_4_Ka_back_color_1, pattern_4_Ka_back_color_2, pattern_4_Ka_back_color_3, pattern_4_Ka_back_color_4, pattern_4_Ka_back);



    texture_map_pattern(pattern_4_Ka_right, CUBE_UV_MAP, pattern_4_Ka);
    pattern_set_transform(pattern_4_Ka, transform_pattern_4_Ka);
Matrix transform_pattern_4_Kd;
    matrix_identity(transform_pattern_4_Kd);
    Pattern pattern_4_Kd = array_of_patterns(7);
    Pattern pattern_4_Kd_right = pattern_4_Kd + 1;
    Pattern pattern_4_Kd_left = pattern_4_Kd + 2;
    Pattern pattern_4_Kd_up = pattern_4_Kd + 3;
    Pattern pattern_4_Kd_down = pattern_4_Kd + 4;
    Pattern pattern_4_Kd_front = pattern_4_Kd + 5;
    Pattern pattern_4_Kd_back = pattern_4_Kd + 6;

    Color pattern_4_Kd_right_color_0_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_4_Kd_right_color_1_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_4_Kd_right_color_2_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_4_Kd_right_color_3_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_4_Kd_right_color_4_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_4_Kd_right_color_0;
    Color pattern_4_Kd_right_color_1;
    Color pattern_4_Kd_right_color_2;
    Color pattern_4_Kd_right_color_3;
    Color pattern_4_Kd_right_color_4;
    color_space_fn(pattern_4_Kd_right_color_0_raw, pattern_4_Kd_right_color_0);
    color_space_fn(pattern_4_Kd_right_color_1_raw, pattern_4_Kd_right_color_1);
    color_space_fn(pattern_4_Kd_right_color_2_raw, pattern_4_Kd_right_color_2);
    color_space_fn(pattern_4_Kd_right_color_3_raw, pattern_4_Kd_right_color_3);
    color_space_fn(pattern_4_Kd_right_color_4_raw, pattern_4_Kd_right_color_4);
    uv_align_check_pattern(pattern_4_Kd_right_color_0, pattern_4_Kd_right_color_1, pattern_4_Kd_right_color_2, pattern_4_Kd_right_color_3, pattern_4_Kd_right_color_4, pattern_4_Kd_right);


    Color pattern_4_Kd_left_color_0_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_4_Kd_left_color_1_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_4_Kd_left_color_2_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_4_Kd_left_color_3_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_4_Kd_left_color_4_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_4_Kd_left_color_0;
    Color pattern_4_Kd_left_color_1;
    Color pattern_4_Kd_left_color_2;
    Color pattern_4_Kd_left_color_3;
    Color pattern_4_Kd_left_color_4;
    color_space_fn(pattern_4_Kd_left_color_0_raw, pattern_4_Kd_left_color_0);
    color_space_fn(pattern_4_Kd_left_color_1_raw, pattern_4_Kd_left_color_1);
    color_space_fn(pattern_4_Kd_left_color_2_raw, pattern_4_Kd_left_color_2);
    color_space_fn(pattern_4_Kd_left_color_3_raw, pattern_4_Kd_left_color_3);
    color_space_fn(pattern_4_Kd_left_color_4_raw, pattern_4_Kd_left_color_4);
    uv_align_check_pattern(pattern_4_Kd_left_color_0, pattern_4_Kd_left_color_1, pattern_4_Kd_left_color_2, pattern_4_Kd_left_color_3, pattern_4_Kd_left_color_4, pattern_4_Kd_left);


    Color pattern_4_Kd_up_color_0_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_4_Kd_up_color_1_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_4_Kd_up_color_2_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_4_Kd_up_color_3_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_4_Kd_up_color_4_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_4_Kd_up_color_0;
    Color pattern_4_Kd_up_color_1;
    Color pattern_4_Kd_up_color_2;
    Color pattern_4_Kd_up_color_3;
    Color pattern_4_Kd_up_color_4;
    color_space_fn(pattern_4_Kd_up_color_0_raw, pattern_4_Kd_up_color_0);
    color_space_fn(pattern_4_Kd_up_color_1_raw, pattern_4_Kd_up_color_1);
    color_space_fn(pattern_4_Kd_up_color_2_raw, pattern_4_Kd_up_color_2);
    color_space_fn(pattern_4_Kd_up_color_3_raw, pattern_4_Kd_up_color_3);
    color_space_fn(pattern_4_Kd_up_color_4_raw, pattern_4_Kd_up_color_4);
    uv_align_check_pattern(pattern_4_Kd_up_color_0, pattern_4_Kd_up_color_1, pattern_4_Kd_up_color_2, pattern_4_Kd_up_color_3, pattern_4_Kd_up_color_4, pattern_4_Kd_up);


    Color pattern_4_Kd_down_color_0_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_4_Kd_down_color_1_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_4_Kd_down_color_2_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_4_Kd_down_color_3_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_4_Kd_down_color_4_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_4_Kd_down_color_0;
    Color pattern_4_Kd_down_color_1;
    Color pattern_4_Kd_down_color_2;
    Color pattern_4_Kd_down_color_3;
    Color pattern_4_Kd_down_color_4;
    color_space_fn(pattern_4_Kd_down_color_0_raw, pattern_4_Kd_down_color_0);
    color_space_fn(pattern_4_Kd_down_color_1_raw, pattern_4_Kd_down_color_1);
    color_space_fn(pattern_4_Kd_down_color_2_raw, pattern_4_Kd_down_color_2);
    color_space_fn(pattern_4_Kd_down_color_3_raw, pattern_4_Kd_down_color_3);
    color_space_fn(pattern_4_Kd_down_color_4_raw, pattern_4_Kd_down_color_4);
    uv_align_check_pattern(pattern_4_Kd_down_color_0, pattern_4_Kd_down_color_1, pattern_4_Kd_down_color_2, pattern_4_Kd_down_color_3, pattern_4_Kd_down_color_4, pattern_4_Kd_down);


    Color pattern_4_Kd_front_color_0_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_4_Kd_front_color_1_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_4_Kd_front_color_2_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_4_Kd_front_color_3_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_4_Kd_front_color_4_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_4_Kd_front_color_0;
    Color pattern_4_Kd_front_color_1;
    Color pattern_4_Kd_front_color_2;
    Color pattern_4_Kd_front_color_3;
    Color pattern_4_Kd_front_color_4;
    color_space_fn(pattern_4_Kd_front_color_0_raw, pattern_4_Kd_front_color_0);
    color_space_fn(pattern_4_Kd_front_color_1_raw, pattern_4_Kd_front_color_1);
    color_space_fn(pattern_4_Kd_front_color_2_raw, pattern_4_Kd_front_color_2);
    color_space_fn(pattern_4_Kd_front_color_3_raw, pattern_4_Kd_front_color_3);
    color_space_fn(pattern_4_Kd_front_color_4_raw, pattern_4_Kd_front_color_4);
    uv_align_check_pattern(pattern_4_Kd_front_color_0, pattern_4_Kd_front_color_1, pattern_4_Kd_front_color_2, pattern_4_Kd_front_color_3, pattern_4_Kd_front_color_4, pattern_4_Kd_front);


    Color pattern_4_Kd_back_color_0_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_4_Kd_back_color_1_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_4_Kd_back_color_2_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_4_Kd_back_color_3_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_4_Kd_back_color_4_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_4_Kd_back_color_0;
    Color pattern_4_Kd_back_color_1;
    Color pattern_4_Kd_back_color_2;
    Color pattern_4_Kd_back_color_3;
    Color pattern_4_Kd_back_color_4;
    color_space_fn(pattern_4_Kd_back_color_0_raw, pattern_4_Kd_back_color_0);
    color_space_fn(pattern_4_Kd_back_color_1_raw, pattern_4_Kd_back_color_1);
    color_space_fn(pattern_4_Kd_back_color_2_raw, pattern_4_Kd_back_color_2);
    color_space_fn(pattern_4_Kd_back_color_3_raw, pattern_4_Kd_back_color_3);
    color_space_fn(pattern_4_Kd_back_color_4_raw, pattern_4_Kd_back_color_4);
    uv_align_check_pattern(pattern_4_Kd_back_color_0, pattern_4_Kd_back_color_1, pattern_4_Kd_back_color_2, pattern_4_Kd_back_color_3, pattern_4_Kd_back_color_4, pattern_4_Kd_back);



    texture_map_pattern(pattern_4_Kd_right, CUBE_UV_MAP, pattern_4_Kd);
    pattern_set_transform(pattern_4_Kd, transform_pattern_4_Kd);
    Pattern pattern_4_Ks = NULL;
    Pattern pattern_4_Ns = NULL;
    Pattern pattern_4_bump = NULL;
    Pattern pattern_4_disp = NULL;
    Pattern pattern_4_refl = NULL;
    Pattern pattern_4_d = NULL;
    Color material_4_color_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color material_4_reflective = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_4_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_4 = material_alloc();
    color_space_fn(material_4_color_raw, material_4->Ka);
    color_space_fn(material_4_color_raw, material_4->Kd);
    color_space_fn(material_4_color_raw, material_4->Ks);
    color_scale(material_4->Ka, 0.2000000000);
    color_scale(material_4->Kd, 0.8000000000);
    color_scale(material_4->Ks, 0.0000000000);
    rgb_to_rgb(material_4_reflective, material_4->refl);
    rgb_to_rgb(material_4_refractive, material_4->Tf);
    material_4->reflective = material_4_reflective[0] > 0.0
                             || material_4_reflective[1] > 0.0
                             || material_4_reflective[2] > 0.0;

    material_4->Tr = 0.0000000000;
    material_4->Ns = 200.0000000000;
    material_4->Ni = 1.0000000000;
    material_4->casts_shadow = true;
    material_set_pattern(material_4, map_Ka, pattern_4_Ka);
    material_set_pattern(material_4, map_Kd, pattern_4_Kd);
    material_set_pattern(material_4, map_Ks, pattern_4_Ks);
    material_set_pattern(material_4, map_Ns, pattern_4_Ns);
    material_set_pattern(material_4, map_d, pattern_4_d);
    material_set_pattern(material_4, map_bump, pattern_4_bump);
    material_set_pattern(material_4, map_disp, pattern_4_disp);
    material_set_pattern(material_4, map_refl, pattern_4_refl);

    Matrix transform_4, transform_4_tmp;
    matrix_identity(transform_4);
    matrix_rotate_y(0.7854000000, transform_4_tmp);
    transform_chain(transform_4_tmp, transform_4);
    matrix_rotate_x(-0.7854000000, transform_4_tmp);
    transform_chain(transform_4_tmp, transform_4);
    matrix_translate(-6.0000000000, -2.0000000000, 0.0000000000, transform_4_tmp);
    transform_chain(transform_4_tmp, transform_4);

    Shape shape_4 = all_shapes + 4;
    cube(shape_4);
    shape_set_material(shape_4, material_4);
    shape_set_transform(shape_4, transform_4);

    /* end shape 4 */
    /* shape 5 */
    
    Matrix transform_pattern_5_Ka;
    matrix_identity(transform_pattern_5_Ka);
    Pattern pattern_5_Ka = array_of_patterns(7);
    Pattern pattern_5_Ka_right = pattern_5_Ka + 1;
    Pattern pattern_5_Ka_left = pattern_5_Ka + 2;
    Pattern pattern_5_Ka_up = pattern_5_Ka + 3;
    Pattern pattern_5_Ka_down = pattern_5_Ka + 4;
    Pattern pattern_5_Ka_front = pattern_5_Ka + 5;
    Pattern pattern_5_Ka_back = pattern_5_Ka + 6;

    Color pattern_5_Ka_right_color_0_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_5_Ka_right_color_1_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_5_Ka_right_color_2_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_5_Ka_right_color_3_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_5_Ka_right_color_4_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_5_Ka_right_color_0;
    Color pattern_5_Ka_right_color_1;
    Color pattern_5_Ka_right_color_2;
    Color pattern_5_Ka_right_color_3;
    Color pattern_5_Ka_right_color_4;
    color_space_fn(pattern_5_Ka_right_color_0_raw, pattern_5_Ka_right_color_0);
    color_space_fn(pattern_5_Ka_right_color_1_raw, pattern_5_Ka_right_color_1);
    color_space_fn(pattern_5_Ka_right_color_2_raw, pattern_5_Ka_right_color_2);
    color_space_fn(pattern_5_Ka_right_color_3_raw, pattern_5_Ka_right_color_3);
    color_space_fn(pattern_5_Ka_right_color_4_raw, pattern_5_Ka_right_color_4);
    uv_align_check_pattern(pattern_5_Ka_right_color_0, pattern_5_Ka_right_color_1, pattern_5_Ka_right_color_2, pattern_5_Ka_right_color_3, pattern_5_Ka_right_color_4, pattern_5_Ka_right);


    Color pattern_5_Ka_left_color_0_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_5_Ka_left_color_1_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_5_Ka_left_color_2_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_5_Ka_left_color_3_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_5_Ka_left_color_4_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_5_Ka_left_color_0;
    Color pattern_5_Ka_left_color_1;
    Color pattern_5_Ka_left_color_2;
    Color pattern_5_Ka_left_color_3;
    Color pattern_5_Ka_left_color_4;
    color_space_fn(pattern_5_Ka_left_color_0_raw, pattern_5_Ka_left_color_0);
    color_space_fn(pattern_5_Ka_left_color_1_raw, pattern_5_Ka_left_color_1);
    color_space_fn(pattern_5_Ka_left_color_2_raw, pattern_5_Ka_left_color_2);
    color_space_fn(pattern_5_Ka_left_color_3_raw, pattern_5_Ka_left_color_3);
    color_space_fn(pattern_5_Ka_left_color_4_raw, pattern_5_Ka_left_color_4);
    uv_align_check_pattern(pattern_5_Ka_left_color_0, pattern_5_Ka_left_color_1, pattern_5_Ka_left_color_2, pattern_5_Ka_left_color_3, pattern_5_Ka_left_color_4, pattern_5_Ka_left);


    Color pattern_5_Ka_up_color_0_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_5_Ka_up_color_1_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_5_Ka_up_color_2_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_5_Ka_up_color_3_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_5_Ka_up_color_4_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_5_Ka_up_color_0;
    Color pattern_5_Ka_up_color_1;
    Color pattern_5_Ka_up_color_2;
    Color pattern_5_Ka_up_color_3;
    Color pattern_5_Ka_up_color_4;
    color_space_fn(pattern_5_Ka_up_color_0_raw, pattern_5_Ka_up_color_0);
    color_space_fn(pattern_5_Ka_up_color_1_raw, pattern_5_Ka_up_color_1);
    color_space_fn(pattern_5_Ka_up_color_2_raw, pattern_5_Ka_up_color_2);
    color_space_fn(pattern_5_Ka_up_color_3_raw, pattern_5_Ka_up_color_3);
    color_space_fn(pattern_5_Ka_up_color_4_raw, pattern_5_Ka_up_color_4);
    uv_align_check_pattern(pattern_5_Ka_up_color_0, pattern_5_Ka_up_color_1, pattern_5_Ka_up_color_2, pattern_5_Ka_up_color_3, pattern_5_Ka_up_color_4, pattern_5_Ka_up);


    Color pattern_5_Ka_down_color_0_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_5_Ka_down_color_1_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_5_Ka_down_color_2_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_5_Ka_down_color_3_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_5_Ka_down_color_4_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_5_Ka_down_color_0;
    Color pattern_5_Ka_down_color_1;
    Color pattern_5_Ka_down_color_2;
    Color pattern_5_Ka_down_color_3;
    Color pattern_5_Ka_down_color_4;
    color_space_fn(pattern_5_Ka_down_color_0_raw, pattern_5_Ka_down_color_0);
    color_space_fn(pattern_5_Ka_down_color_1_raw, pattern_5_Ka_down_color_1);
    color_space_fn(pattern_5_Ka_down_color_2_raw, pattern_5_Ka_down_color_2);
    color_space_fn(pattern_5_Ka_down_color_3_raw, pattern_5_Ka_down_color_3);
    color_space_fn(pattern_5_Ka_down_color_4_raw, pattern_5_Ka_down_color_4);
    uv_align_check_pattern(pattern_5_Ka_down_color_0, pattern_5_Ka_down_color_1, pattern_5_Ka_down_color_2, pattern_5_Ka_down_color_3, pattern_5_Ka_down_color_4, pattern_5_Ka_down);


    Color pattern_5_Ka_front_color_0_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_5_Ka_front_color_1_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_5_Ka_front_color_2_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_5_Ka_front_color_3_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_5_Ka_front_color_4_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_5_Ka_front_color_0;
    Color pattern_5_Ka_front_color_1;
    Color pattern_5_Ka_front_color_2;
    Color pattern_5_Ka_front_color_3;
    Color pattern_5_Ka_front_color_4;
    color_space_fn(pattern_5_Ka_front_color_0_raw, pattern_5_Ka_front_color_0);
    color_space_fn(pattern_5_Ka_front_color_1_raw, pattern_5_Ka_front_color_1);
    color_space_fn(pattern_5_Ka_front_color_2_raw, pattern_5_Ka_front_color_2);
    color_space_fn(pattern_5_Ka_front_color_3_raw, pattern_5_Ka_front_color_3);
    color_space_fn(pattern_5_Ka_front_color_4_raw, pattern_5_Ka_front_color_4);
    uv_align_check_pattern(pattern_5_Ka_front_color_0, pattern_5_Ka_front_color_1, pattern_5_Ka_front_color_2, pattern_5_Ka_front_color_3, pattern_5_Ka_front_color_4, pattern_5_Ka_front);


    Color pattern_5_Ka_back_color_0_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_5_Ka_back_color_1_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_5_Ka_back_color_2_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_5_Ka_back_color_3_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_5_Ka_back_color_4_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_5_Ka_back_color_0;
    Color pattern_5_Ka_back_color_1;
    Color pattern_5_Ka_back_color_2;
    Color pattern_5_Ka_back_color_3;
    Color pattern_5_Ka_back_color_4;
    color_space_fn(pattern_5_Ka_back_color_0_raw, pattern_5_Ka_back_color_0);
    color_space_fn(pattern_5_Ka_back_color_1_raw, pattern_5_Ka_back_color_1);
    color_space_fn(pattern_5_Ka_back_color_2_raw, pattern_5_Ka_back_color_2);
    color_space_fn(pattern_5_Ka_back_color_3_raw, pattern_5_Ka_back_color_3);
    color_space_fn(pattern_5_Ka_back_color_4_raw, pattern_5_Ka_back_color_4);
    uv_align_check_pattern(pattern_5_Ka_back_color_0, pattern_5_Ka_back_color_1, pattern_5_Ka_back_color_2, pattern_5_Ka_back_color_3, pattern_5_Ka_back_color_4, pattern_5_Ka_back);



    texture_map_pattern(pattern_5_Ka_right, CUBE_UV_MAP, pattern_5_Ka);
    pattern_set_transform(pattern_5_Ka, transform_pattern_5_Ka);
Matrix transform_pattern_5_Kd;
    matrix_identity(transform_pattern_5_Kd);
    Pattern pattern_5_Kd = array_of_patterns(7);
    Pattern pattern_5_Kd_right = pattern_5_Kd + 1;
    Pattern pattern_5_Kd_left = pattern_5_Kd + 2;
    Pattern pattern_5_Kd_up = pattern_5_Kd + 3;
    Pattern pattern_5_Kd_down = pattern_5_Kd + 4;
    Pattern pattern_5_Kd_front = pattern_5_Kd + 5;
    Pattern pattern_5_Kd_back = pattern_5_Kd + 6;

    Color pattern_5_Kd_right_color_0_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_5_Kd_right_color_1_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_5_Kd_right_color_2_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_5_Kd_right_color_3_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_5_Kd_right_color_4_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_5_Kd_right_color_0;
    Color pattern_5_Kd_right_color_1;
    Color pattern_5_Kd_right_color_2;
    Color pattern_5_Kd_right_color_3;
    Color pattern_5_Kd_right_color_4;
    color_space_fn(pattern_5_Kd_right_color_0_raw, pattern_5_Kd_right_color_0);
    color_space_fn(pattern_5_Kd_right_color_1_raw, pattern_5_Kd_right_color_1);
    color_space_fn(pattern_5_Kd_right_color_2_raw, pattern_5_Kd_right_color_2);
    color_space_fn(pattern_5_Kd_right_color_3_raw, pattern_5_Kd_right_color_3);
    color_space_fn(pattern_5_Kd_right_color_4_raw, pattern_5_Kd_right_color_4);
    uv_align_check_pattern(pattern_5_Kd_right_color_0, pattern_5_Kd_right_color_1, pattern_5_Kd_right_color_2, pattern_5_Kd_right_color_3, pattern_5_Kd_right_color_4, pattern_5_Kd_right);


    Color pattern_5_Kd_left_color_0_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_5_Kd_left_color_1_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_5_Kd_left_color_2_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_5_Kd_left_color_3_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_5_Kd_left_color_4_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_5_Kd_left_color_0;
    Color pattern_5_Kd_left_color_1;
    Color pattern_5_Kd_left_color_2;
    Color pattern_5_Kd_left_color_3;
    Color pattern_5_Kd_left_color_4;
    color_space_fn(pattern_5_Kd_left_color_0_raw, pattern_5_Kd_left_color_0);
    color_space_fn(pattern_5_Kd_left_color_1_raw, pattern_5_Kd_left_color_1);
    color_space_fn(pattern_5_Kd_left_color_2_raw, pattern_5_Kd_left_color_2);
    color_space_fn(pattern_5_Kd_left_color_3_raw, pattern_5_Kd_left_color_3);
    color_space_fn(pattern_5_Kd_left_color_4_raw, pattern_5_Kd_left_color_4);
    uv_align_check_pattern(pattern_5_Kd_left_color_0, pattern_5_Kd_left_color_1, pattern_5_Kd_left_color_2, pattern_5_Kd_left_color_3, pattern_5_Kd_left_color_4, pattern_5_Kd_left);


    Color pattern_5_Kd_up_color_0_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_5_Kd_up_color_1_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_5_Kd_up_color_2_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_5_Kd_up_color_3_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_5_Kd_up_color_4_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_5_Kd_up_color_0;
    Color pattern_5_Kd_up_color_1;
    Color pattern_5_Kd_up_color_2;
    Color pattern_5_Kd_up_color_3;
    Color pattern_5_Kd_up_color_4;
    color_space_fn(pattern_5_Kd_up_color_0_raw, pattern_5_Kd_up_color_0);
    color_space_fn(pattern_5_Kd_up_color_1_raw, pattern_5_Kd_up_color_1);
    color_space_fn(pattern_5_Kd_up_color_2_raw, pattern_5_Kd_up_color_2);
    color_space_fn(pattern_5_Kd_up_color_3_raw, pattern_5_Kd_up_color_3);
    color_space_fn(pattern_5_Kd_up_color_4_raw, pattern_5_Kd_up_color_4);
    uv_align_check_pattern(pattern_5_Kd_up_color_0, pattern_5_Kd_up_color_1, pattern_5_Kd_up_color_2, pattern_5_Kd_up_color_3, pattern_5_Kd_up_color_4, pattern_5_Kd_up);


    Color pattern_5_Kd_down_color_0_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_5_Kd_down_color_1_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_5_Kd_down_color_2_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_5_Kd_down_color_3_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_5_Kd_down_color_4_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_5_Kd_down_color_0;
    Color pattern_5_Kd_down_color_1;
    Color pattern_5_Kd_down_color_2;
    Color pattern_5_Kd_down_color_3;
    Color pattern_5_Kd_down_color_4;
    color_space_fn(pattern_5_Kd_down_color_0_raw, pattern_5_Kd_down_color_0);
    color_space_fn(pattern_5_Kd_down_color_1_raw, pattern_5_Kd_down_color_1);
    color_space_fn(pattern_5_Kd_down_color_2_raw, pattern_5_Kd_down_color_2);
    color_space_fn(pattern_5_Kd_down_color_3_raw, pattern_5_Kd_down_color_3);
    color_space_fn(pattern_5_Kd_down_color_4_raw, pattern_5_Kd_down_color_4);
    uv_align_check_pattern(pattern_5_Kd_down_color_0, pattern_5_Kd_down_color_1, pattern_5_Kd_down_color_2, pattern_5_Kd_down_color_3, pattern_5_Kd_down_color_4, pattern_5_Kd_down);


    Color pattern_5_Kd_front_color_0_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_5_Kd_front_color_1_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_5_Kd_front_color_2_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_5_Kd_front_color_3_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_5_Kd_front_color_4_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_5_Kd_front_color_0;
    Color pattern_5_Kd_front_color_1;
    Color pattern_5_Kd_front_color_2;
    Color pattern_5_Kd_front_color_3;
    Color pattern_5_Kd_front_color_4;
    color_space_fn(pattern_5_Kd_front_color_0_raw, pattern_5_Kd_front_color_0);
    color_space_fn(pattern_5_Kd_front_color_1_raw, pattern_5_Kd_front_color_1);
    color_space_fn(pattern_5_Kd_front_color_2_raw, pattern_5_Kd_front_color_2);
    color_space_fn(pattern_5_Kd_front_color_3_raw, pattern_5_Kd_front_color_3);
    color_space_fn(pattern_5_Kd_front_color_4_raw, pattern_5_Kd_front_color_4);
    uv_align_check_pattern(pattern_5_Kd_front_color_0, pattern_5_Kd_front_color_1, pattern_5_Kd_front_color_2, pattern_5_Kd_front_color_3, pattern_5_Kd_front_color_4, pattern_5_Kd_front);


    Color pattern_5_Kd_back_color_0_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_5_Kd_back_color_1_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_5_Kd_back_color_2_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_5_Kd_back_color_3_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_5_Kd_back_color_4_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_5_Kd_back_color_0;
    Color pattern_5_Kd_back_color_1;
    Color pattern_5_Kd_back_color_2;
    Color pattern_5_Kd_back_color_3;
    Color pattern_5_Kd_back_color_4;
    color_space_fn(pattern_5_Kd_back_color_0_raw, pattern_5_Kd_back_color_0);
    color_space_fn(pattern_5_Kd_back_color_1_raw, pattern_5_Kd_back_color_1);
    color_space_fn(pattern_5_Kd_back_color_2_raw, pattern_5_Kd_back_color_2);
    color_space_fn(pattern_5_Kd_back_color_3_raw, pattern_5_Kd_back_color_3);
    color_space_fn(pattern_5_Kd_back_color_4_raw, pattern_5_Kd_back_color_4);
    uv_align_check_pattern(pattern_5_Kd_back_color_0, pattern_5_Kd_back_color_1, pattern_5_Kd_back_color_2, pattern_5_Kd_back_color_3, pattern_5_Kd_back_color_4, pattern_5_Kd_back);



    texture_map_pattern(pattern_5_Kd_right, CUBE_UV_MAP, pattern_5_Kd);
    pattern_set_transform(pattern_5_Kd, transform_pattern_5_Kd);
    Pattern pattern_5_Ks = NULL;
    Pattern pattern_5_Ns = NULL;
    Pattern pattern_5_bump = NULL;
    Pattern pattern_5_disp = NULL;
    Pattern pattern_5_refl = NULL;
    Pattern pattern_5_d = NULL;
    Color material_5_color_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color material_5_reflective = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_5_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_5 = material_alloc();
    color_space_fn(material_5_color_raw, material_5->Ka);
    color_space_fn(material_5_color_raw, material_5->Kd);
    color_space_fn(material_5_color_raw, material_5->Ks);
    color_scale(material_5->Ka, 0.2000000000);
    color_scale(material_5->Kd, 0.8000000000);
    color_scale(material_5->Ks, 0.0000000000);
    rgb_to_rgb(material_5_reflective, material_5->refl);
    rgb_to_rgb(material_5_refractive, material_5->Tf);
    material_5->reflective = material_5_reflective[0] > 0.0
                             || material_5_reflective[1] > 0.0
                             || material_5_reflective[2] > 0.0;

    material_5->Tr = 0.0000000000;
    material_5->Ns = 200.0000000000;
    material_5->Ni = 1.0000000000;
    material_5->casts_shadow = true;
    material_set_pattern(material_5, map_Ka, pattern_5_Ka);
    material_set_pattern(material_5, map_Kd, pattern_5_Kd);
    material_set_pattern(material_5, map_Ks, pattern_5_Ks);
    material_set_pattern(material_5, map_Ns, pattern_5_Ns);
    material_set_pattern(material_5, map_d, pattern_5_d);
    material_set_pattern(material_5, map_bump, pattern_5_bump);
    material_set_pattern(material_5, map_disp, pattern_5_disp);
    material_set_pattern(material_5, map_refl, pattern_5_refl);

    Matrix transform_5, transform_5_tmp;
    matrix_identity(transform_5);
    matrix_rotate_y(2.3562000000, transform_5_tmp);
    transform_chain(transform_5_tmp, transform_5);
    matrix_rotate_x(-0.7854000000, transform_5_tmp);
    transform_chain(transform_5_tmp, transform_5);
    matrix_translate(-2.0000000000, -2.0000000000, 0.0000000000, transform_5_tmp);
    transform_chain(transform_5_tmp, transform_5);

    Shape shape_5 = all_shapes + 5;
    cube(shape_5);
    shape_set_material(shape_5, material_5);
    shape_set_transform(shape_5, transform_5);

    /* end shape 5 */
    /* shape 6 */
    
    Matrix transform_pattern_6_Ka;
    matrix_identity(transform_pattern_6_Ka);
    Pattern pattern_6_Ka = array_of_patterns(7);
    Pattern pattern_6_Ka_right = pattern_6_Ka + 1;
    Pattern pattern_6_Ka_left = pattern_6_Ka + 2;
    Pattern pattern_6_Ka_up = pattern_6_Ka + 3;
    Pattern pattern_6_Ka_down = pattern_6_Ka + 4;
    Pattern pattern_6_Ka_front = pattern_6_Ka + 5;
    Pattern pattern_6_Ka_back = pattern_6_Ka + 6;

    Color pattern_6_Ka_right_color_0_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_6_Ka_right_color_1_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_6_Ka_right_color_2_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_6_Ka_right_color_3_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_6_Ka_right_color_4_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_6_Ka_right_color_0;
    Color pattern_6_Ka_right_color_1;
    Color pattern_6_Ka_right_color_2;
    Color pattern_6_Ka_right_color_3;
    Color pattern_6_Ka_right_color_4;
    color_space_fn(pattern_6_Ka_right_color_0_raw, pattern_6_Ka_right_color_0);
    color_space_fn(pattern_6_Ka_right_color_1_raw, pattern_6_Ka_right_color_1);
    color_space_fn(pattern_6_Ka_right_color_2_raw, pattern_6_Ka_right_color_2);
    color_space_fn(pattern_6_Ka_right_color_3_raw, pattern_6_Ka_right_color_3);
    color_space_fn(pattern_6_Ka_right_color_4_raw, pattern_6_Ka_right_color_4);
    uv_align_check_pattern(pattern_6_Ka_right_color_0, pattern_6_Ka_right_color_1, pattern_6_Ka_right_color_2, pattern_6_Ka_right_color_3, pattern_6_Ka_right_color_4, pattern_6_Ka_right);


    Color pattern_6_Ka_left_color_0_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_6_Ka_left_color_1_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_6_Ka_left_color_2_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_6_Ka_left_color_3_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_6_Ka_left_color_4_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_6_Ka_left_color_0;
    Color pattern_6_Ka_left_color_1;
    Color pattern_6_Ka_left_color_2;
    Color pattern_6_Ka_left_color_3;
    Color pattern_6_Ka_left_color_4;
    color_space_fn(pattern_6_Ka_left_color_0_raw, pattern_6_Ka_left_color_0);
    color_space_fn(pattern_6_Ka_left_color_1_raw, pattern_6_Ka_left_color_1);
    color_space_fn(pattern_6_Ka_left_color_2_raw, pattern_6_Ka_left_color_2);
    color_space_fn(pattern_6_Ka_left_color_3_raw, pattern_6_Ka_left_color_3);
    color_space_fn(pattern_6_Ka_left_color_4_raw, pattern_6_Ka_left_color_4);
    uv_align_check_pattern(pattern_6_Ka_left_color_0, pattern_6_Ka_left_color_1, pattern_6_Ka_left_color_2, pattern_6_Ka_left_color_3, pattern_6_Ka_left_color_4, pattern_6_Ka_left);


    Color pattern_6_Ka_up_color_0_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_6_Ka_up_color_1_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_6_Ka_up_color_2_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_6_Ka_up_color_3_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_6_Ka_up_color_4_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_6_Ka_up_color_0;
    Color pattern_6_Ka_up_color_1;
    Color pattern_6_Ka_up_color_2;
    Color pattern_6_Ka_up_color_3;
    Color pattern_6_Ka_up_color_4;
    color_space_fn(pattern_6_Ka_up_color_0_raw, pattern_6_Ka_up_color_0);
    color_space_fn(pattern_6_Ka_up_color_1_raw, pattern_6_Ka_up_color_1);
    color_space_fn(pattern_6_Ka_up_color_2_raw, pattern_6_Ka_up_color_2);
    color_space_fn(pattern_6_Ka_up_color_3_raw, pattern_6_Ka_up_color_3);
    color_space_fn(pattern_6_Ka_up_color_4_raw, pattern_6_Ka_up_color_4);
    uv_align_check_pattern(pattern_6_Ka_up_color_0, pattern_6_Ka_up_color_1, pattern_6_Ka_up_color_2, pattern_6_Ka_up_color_3, pattern_6_Ka_up_color_4, pattern_6_Ka_up);


    Color pattern_6_Ka_down_color_0_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_6_Ka_down_color_1_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_6_Ka_down_color_2_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_6_Ka_down_color_3_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_6_Ka_down_color_4_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_6_Ka_down_color_0;
    Color pattern_6_Ka_down_color_1;
    Color pattern_6_Ka_down_color_2;
    Color pattern_6_Ka_down_color_3;
    Color pattern_6_Ka_down_color_4;
    color_space_fn(pattern_6_Ka_down_color_0_raw, pattern_6_Ka_down_color_0);
    color_space_fn(pattern_6_Ka_down_color_1_raw, pattern_6_Ka_down_color_1);
    color_space_fn(pattern_6_Ka_down_color_2_raw, pattern_6_Ka_down_color_2);
    color_space_fn(pattern_6_Ka_down_color_3_raw, pattern_6_Ka_down_color_3);
    color_space_fn(pattern_6_Ka_down_color_4_raw, pattern_6_Ka_down_color_4);
    uv_align_check_pattern(pattern_6_Ka_down_color_0, pattern_6_Ka_down_color_1, pattern_6_Ka_down_color_2, pattern_6_Ka_down_color_3, pattern_6_Ka_down_color_4, pattern_6_Ka_down);


    Color pattern_6_Ka_front_color_0_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_6_Ka_front_color_1_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_6_Ka_front_color_2_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_6_Ka_front_color_3_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_6_Ka_front_color_4_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_6_Ka_front_color_0;
    Color pattern_6_Ka_front_color_1;
    Color pattern_6_Ka_front_color_2;
    Color pattern_6_Ka_front_color_3;
    Color pattern_6_Ka_front_color_4;
    color_space_fn(pattern_6_Ka_front_color_0_raw, pattern_6_Ka_front_color_0);
    color_space_fn(pattern_6_Ka_front_color_1_raw, pattern_6_Ka_front_color_1);
    color_space_fn(pattern_6_Ka_front_color_2_raw, pattern_6_Ka_front_color_2);
    color_space_fn(pattern_6_Ka_front_color_3_raw, pattern_6_Ka_front_color_3);
    color_space_fn(pattern_6_Ka_front_color_4_raw, pattern_6_Ka_front_color_4);
    uv_align_check_pattern(pattern_6_Ka_front_color_0, pattern_6_Ka_front_color_1, pattern_6_Ka_front_color_2, pattern_6_Ka_front_color_3, pattern_6_Ka_front_color_4, pattern_6_Ka_front);


    Color pattern_6_Ka_back_color_0_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_6_Ka_back_color_1_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_6_Ka_back_color_2_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_6_Ka_back_color_3_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_6_Ka_back_color_4_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_6_Ka_back_color_0;
    Color pattern_6_Ka_back_color_1;
    Color pattern_6_Ka_back_color_2;
    Color pattern_6_Ka_back_color_3;
    Color pattern_6_Ka_back_color_4;
    color_space_fn(pattern_6_Ka_back_color_0_raw, pattern_6_Ka_back_color_0);
    color_space_fn(pattern_6_Ka_back_color_1_raw, pattern_6_Ka_back_color_1);
    color_space_fn(pattern_6_Ka_back_color_2_raw, pattern_6_Ka_back_color_2);
    color_space_fn(pattern_6_Ka_back_color_3_raw, pattern_6_Ka_back_color_3);
    color_space_fn(pattern_6_Ka_back_color_4_raw, pattern_6_Ka_back_color_4);
    uv_align_check_pattern(pattern_6_Ka_back_color_0, pattern_6_Ka_back_color_1, pattern_6_Ka_back_color_2, pattern_6_Ka_back_color_3, pattern_6_Ka_back_color_4, pattern_6_Ka_back);



    texture_map_pattern(pattern_6_Ka_right, CUBE_UV_MAP, pattern_6_Ka);
    pattern_set_transform(pattern_6_Ka, transform_pattern_6_Ka);
Matrix transform_pattern_6_Kd;
    matrix_identity(transform_pattern_6_Kd);
    Pattern pattern_6_Kd = array_of_patterns(7);
    Pattern pattern_6_Kd_right = pattern_6_Kd + 1;
    Pattern pattern_6_Kd_left = pattern_6_Kd + 2;
    Pattern pattern_6_Kd_up = pattern_6_Kd + 3;
    Pattern pattern_6_Kd_down = pattern_6_Kd + 4;
    Pattern pattern_6_Kd_front = pattern_6_Kd + 5;
    Pattern pattern_6_Kd_back = pattern_6_Kd + 6;

    Color pattern_6_Kd_right_color_0_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_6_Kd_right_color_1_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_6_Kd_right_color_2_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_6_Kd_right_color_3_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_6_Kd_right_color_4_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_6_Kd_right_color_0;
    Color pattern_6_Kd_right_color_1;
    Color pattern_6_Kd_right_color_2;
    Color pattern_6_Kd_right_color_3;
    Color pattern_6_Kd_right_color_4;
    color_space_fn(pattern_6_Kd_right_color_0_raw, pattern_6_Kd_right_color_0);
    color_space_fn(pattern_6_Kd_right_color_1_raw, pattern_6_Kd_right_color_1);
    color_space_fn(pattern_6_Kd_right_color_2_raw, pattern_6_Kd_right_color_2);
    color_space_fn(pattern_6_Kd_right_color_3_raw, pattern_6_Kd_right_color_3);
    color_space_fn(pattern_6_Kd_right_color_4_raw, pattern_6_Kd_right_color_4);
    uv_align_check_pattern(pattern_6_Kd_right_color_0, pattern_6_Kd_right_color_1, pattern_6_Kd_right_color_2, pattern_6_Kd_right_color_3, pattern_6_Kd_right_color_4, pattern_6_Kd_right);


    Color pattern_6_Kd_left_color_0_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_6_Kd_left_color_1_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_6_Kd_left_color_2_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_6_Kd_left_color_3_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_6_Kd_left_color_4_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_6_Kd_left_color_0;
    Color pattern_6_Kd_left_color_1;
    Color pattern_6_Kd_left_color_2;
    Color pattern_6_Kd_left_color_3;
    Color pattern_6_Kd_left_color_4;
    color_space_fn(pattern_6_Kd_left_color_0_raw, pattern_6_Kd_left_color_0);
    color_space_fn(pattern_6_Kd_left_color_1_raw, pattern_6_Kd_left_color_1);
    color_space_fn(pattern_6_Kd_left_color_2_raw, pattern_6_Kd_left_color_2);
    color_space_fn(pattern_6_Kd_left_color_3_raw, pattern_6_Kd_left_color_3);
    color_space_fn(pattern_6_Kd_left_color_4_raw, pattern_6_Kd_left_color_4);
    uv_align_check_pattern(pattern_6_Kd_left_color_0, pattern_6_Kd_left_color_1, pattern_6_Kd_left_color_2, pattern_6_Kd_left_color_3, pattern_6_Kd_left_color_4, pattern_6_Kd_left);


    Color pattern_6_Kd_up_color_0_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_6_Kd_up_color_1_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_6_Kd_up_color_2_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_6_Kd_up_color_3_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_6_Kd_up_color_4_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_6_Kd_up_color_0;
    Color pattern_6_Kd_up_color_1;
    Color pattern_6_Kd_up_color_2;
    Color pattern_6_Kd_up_color_3;
    Color pattern_6_Kd_up_color_4;
    color_space_fn(pattern_6_Kd_up_color_0_raw, pattern_6_Kd_up_color_0);
    color_space_fn(pattern_6_Kd_up_color_1_raw, pattern_6_Kd_up_color_1);
    color_space_fn(pattern_6_Kd_up_color_2_raw, pattern_6_Kd_up_color_2);
    color_space_fn(pattern_6_Kd_up_color_3_raw, pattern_6_Kd_up_color_3);
    color_space_fn(pattern_6_Kd_up_color_4_raw, pattern_6_Kd_up_color_4);
    uv_align_check_pattern(pattern_6_Kd_up_color_0, pattern_6_Kd_up_color_1, pattern_6_Kd_up_color_2, pattern_6_Kd_up_color_3, pattern_6_Kd_up_color_4, pattern_6_Kd_up);


    Color pattern_6_Kd_down_color_0_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_6_Kd_down_color_1_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_6_Kd_down_color_2_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_6_Kd_down_color_3_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_6_Kd_down_color_4_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_6_Kd_down_color_0;
    Color pattern_6_Kd_down_color_1;
    Color pattern_6_Kd_down_color_2;
    Color pattern_6_Kd_down_color_3;
    Color pattern_6_Kd_down_color_4;
    color_space_fn(pattern_6_Kd_down_color_0_raw, pattern_6_Kd_down_color_0);
    color_space_fn(pattern_6_Kd_down_color_1_raw, pattern_6_Kd_down_color_1);
    color_space_fn(pattern_6_Kd_down_color_2_raw, pattern_6_Kd_down_color_2);
    color_space_fn(pattern_6_Kd_down_color_3_raw, pattern_6_Kd_down_color_3);
    color_space_fn(pattern_6_Kd_down_color_4_raw, pattern_6_Kd_down_color_4);
    uv_align_check_pattern(pattern_6_Kd_down_color_0, pattern_6_Kd_down_color_1, pattern_6_Kd_down_color_2, pattern_6_Kd_down_color_3, pattern_6_Kd_down_color_4, pattern_6_Kd_down);


    Color pattern_6_Kd_front_color_0_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_6_Kd_front_color_1_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_6_Kd_front_color_2_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_6_Kd_front_color_3_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_6_Kd_front_color_4_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_6_Kd_front_color_0;
    Color pattern_6_Kd_front_color_1;
    Color pattern_6_Kd_front_color_2;
    Color pattern_6_Kd_front_color_3;
    Color pattern_6_Kd_front_color_4;
    color_space_fn(pattern_6_Kd_front_color_0_raw, pattern_6_Kd_front_color_0);
    color_space_fn(pattern_6_Kd_front_color_1_raw, pattern_6_Kd_front_color_1);
    color_space_fn(pattern_6_Kd_front_color_2_raw, pattern_6_Kd_front_color_2);
    color_space_fn(pattern_6_Kd_front_color_3_raw, pattern_6_Kd_front_color_3);
    color_space_fn(pattern_6_Kd_front_color_4_raw, pattern_6_Kd_front_color_4);
    uv_align_check_pattern(pattern_6_Kd_front_color_0, pattern_6_Kd_front_color_1, pattern_6_Kd_front_color_2, pattern_6_Kd_front_color_3, pattern_6_Kd_front_color_4, pattern_6_Kd_front);


    Color pattern_6_Kd_back_color_0_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_6_Kd_back_color_1_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_6_Kd_back_color_2_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_6_Kd_back_color_3_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_6_Kd_back_color_4_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_6_Kd_back_color_0;
    Color pattern_6_Kd_back_color_1;
    Color pattern_6_Kd_back_color_2;
    Color pattern_6_Kd_back_color_3;
    Color pattern_6_Kd_back_color_4;
    color_space_fn(pattern_6_Kd_back_color_0_raw, pattern_6_Kd_back_color_0);
    color_space_fn(pattern_6_Kd_back_color_1_raw, pattern_6_Kd_back_color_1);
    color_space_fn(pattern_6_Kd_back_color_2_raw, pattern_6_Kd_back_color_2);
    color_space_fn(pattern_6_Kd_back_color_3_raw, pattern_6_Kd_back_color_3);
    color_space_fn(pattern_6_Kd_back_color_4_raw, pattern_6_Kd_back_color_4);
    uv_align_check_pattern(pattern_6_Kd_back_color_0, pattern_6_Kd_back_color_1, pattern_6_Kd_back_color_2, pattern_6_Kd_back_color_3, pattern_6_Kd_back_color_4, pattern_6_Kd_back);



    texture_map_pattern(pattern_6_Kd_right, CUBE_UV_MAP, pattern_6_Kd);
    pattern_set_transform(pattern_6_Kd, transform_pattern_6_Kd);
    Pattern pattern_6_Ks = NULL;
    Pattern pattern_6_Ns = NULL;
    Pattern pattern_6_bump = NULL;
    Pattern pattern_6_disp = NULL;
    Pattern pattern_6_refl = NULL;
    Pattern pattern_6_d = NULL;
    Color material_6_color_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color material_6_reflective = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_6_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_6 = material_alloc();
    color_space_fn(material_6_color_raw, material_6->Ka);
    color_space_fn(material_6_color_raw, material_6->Kd);
    color_space_fn(material_6_color_raw, material_6->Ks);
    color_scale(material_6->Ka, 0.2000000000);
    color_scale(material_6->Kd, 0.8000000000);
    color_scale(material_6->Ks, 0.0000000000);
    rgb_to_rgb(material_6_reflective, material_6->refl);
    rgb_to_rgb(material_6_refractive, material_6->Tf);
    material_6->reflective = material_6_reflective[0] > 0.0
                             || material_6_reflective[1] > 0.0
                             || material_6_reflective[2] > 0.0;

    material_6->Tr = 0.0000000000;
    material_6->Ns = 200.0000000000;
    material_6->Ni = 1.0000000000;
    material_6->casts_shadow = true;
    material_set_pattern(material_6, map_Ka, pattern_6_Ka);
    material_set_pattern(material_6, map_Kd, pattern_6_Kd);
    material_set_pattern(material_6, map_Ks, pattern_6_Ks);
    material_set_pattern(material_6, map_Ns, pattern_6_Ns);
    material_set_pattern(material_6, map_d, pattern_6_d);
    material_set_pattern(material_6, map_bump, pattern_6_bump);
    material_set_pattern(material_6, map_disp, pattern_6_disp);
    material_set_pattern(material_6, map_refl, pattern_6_refl);

    Matrix transform_6, transform_6_tmp;
    matrix_identity(transform_6);
    matrix_rotate_y(3.9270000000, transform_6_tmp);
    transform_chain(transform_6_tmp, transform_6);
    matrix_rotate_x(-0.7854000000, transform_6_tmp);
    transform_chain(transform_6_tmp, transform_6);
    matrix_translate(2.0000000000, -2.0000000000, 0.0000000000, transform_6_tmp);
    transform_chain(transform_6_tmp, transform_6);

    Shape shape_6 = all_shapes + 6;
    cube(shape_6);
    shape_set_material(shape_6, material_6);
    shape_set_transform(shape_6, transform_6);

    /* end shape 6 */
    /* shape 7 */
    
    Matrix transform_pattern_7_Ka;
    matrix_identity(transform_pattern_7_Ka);
    Pattern pattern_7_Ka = array_of_patterns(7);
    Pattern pattern_7_Ka_right = pattern_7_Ka + 1;
    Pattern pattern_7_Ka_left = pattern_7_Ka + 2;
    Pattern pattern_7_Ka_up = pattern_7_Ka + 3;
    Pattern pattern_7_Ka_down = pattern_7_Ka + 4;
    Pattern pattern_7_Ka_front = pattern_7_Ka + 5;
    Pattern pattern_7_Ka_back = pattern_7_Ka + 6;

    Color pattern_7_Ka_right_color_0_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_7_Ka_right_color_1_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_7_Ka_right_color_2_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_7_Ka_right_color_3_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_7_Ka_right_color_4_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_7_Ka_right_color_0;
    Color pattern_7_Ka_right_color_1;
    Color pattern_7_Ka_right_color_2;
    Color pattern_7_Ka_right_color_3;
    Color pattern_7_Ka_right_color_4;
    color_space_fn(pattern_7_Ka_right_color_0_raw, pattern_7_Ka_right_color_0);
    color_space_fn(pattern_7_Ka_right_color_1_raw, pattern_7_Ka_right_color_1);
    color_space_fn(pattern_7_Ka_right_color_2_raw, pattern_7_Ka_right_color_2);
    color_space_fn(pattern_7_Ka_right_color_3_raw, pattern_7_Ka_right_color_3);
    color_space_fn(pattern_7_Ka_right_color_4_raw, pattern_7_Ka_right_color_4);
    uv_align_check_pattern(pattern_7_Ka_right_color_0, pattern_7_Ka_right_color_1, pattern_7_Ka_right_color_2, pattern_7_Ka_right_color_3, pattern_7_Ka_right_color_4, pattern_7_Ka_right);


    Color pattern_7_Ka_left_color_0_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_7_Ka_left_color_1_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_7_Ka_left_color_2_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_7_Ka_left_color_3_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_7_Ka_left_color_4_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_7_Ka_left_color_0;
    Color pattern_7_Ka_left_color_1;
    Color pattern_7_Ka_left_color_2;
    Color pattern_7_Ka_left_color_3;
    Color pattern_7_Ka_left_color_4;
    color_space_fn(pattern_7_Ka_left_color_0_raw, pattern_7_Ka_left_color_0);
    color_space_fn(pattern_7_Ka_left_color_1_raw, pattern_7_Ka_left_color_1);
    color_space_fn(pattern_7_Ka_left_color_2_raw, pattern_7_Ka_left_color_2);
    color_space_fn(pattern_7_Ka_left_color_3_raw, pattern_7_Ka_left_color_3);
    color_space_fn(pattern_7_Ka_left_color_4_raw, pattern_7_Ka_left_color_4);
    uv_align_check_pattern(pattern_7_Ka_left_color_0, pattern_7_Ka_left_color_1, pattern_7_Ka_left_color_2, pattern_7_Ka_left_color_3, pattern_7_Ka_left_color_4, pattern_7_Ka_left);


    Color pattern_7_Ka_up_color_0_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_7_Ka_up_color_1_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_7_Ka_up_color_2_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_7_Ka_up_color_3_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_7_Ka_up_color_4_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_7_Ka_up_color_0;
    Color pattern_7_Ka_up_color_1;
    Color pattern_7_Ka_up_color_2;
    Color pattern_7_Ka_up_color_3;
    Color pattern_7_Ka_up_color_4;
    color_space_fn(pattern_7_Ka_up_color_0_raw, pattern_7_Ka_up_color_0);
    color_space_fn(pattern_7_Ka_up_color_1_raw, pattern_7_Ka_up_color_1);
    color_space_fn(pattern_7_Ka_up_color_2_raw, pattern_7_Ka_up_color_2);
    color_space_fn(pattern_7_Ka_up_color_3_raw, pattern_7_Ka_up_color_3);
    color_space_fn(pattern_7_Ka_up_color_4_raw, pattern_7_Ka_up_color_4);
    uv_align_check_pattern(pattern_7_Ka_up_color_0, pattern_7_Ka_up_color_1, pattern_7_Ka_up_color_2, pattern_7_Ka_up_color_3, pattern_7_Ka_up_color_4, pattern_7_Ka_up);


    Color pattern_7_Ka_down_color_0_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_7_Ka_down_color_1_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_7_Ka_down_color_2_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_7_Ka_down_color_3_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_7_Ka_down_color_4_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_7_Ka_down_color_0;
    Color pattern_7_Ka_down_color_1;
    Color pattern_7_Ka_down_color_2;
    Color pattern_7_Ka_down_color_3;
    Color pattern_7_Ka_down_color_4;
    color_space_fn(pattern_7_Ka_down_color_0_raw, pattern_7_Ka_down_color_0);
    color_space_fn(pattern_7_Ka_down_color_1_raw, pattern_7_Ka_down_color_1);
    color_space_fn(pattern_7_Ka_down_color_2_raw, pattern_7_Ka_down_color_2);
    color_space_fn(pattern_7_Ka_down_color_3_raw, pattern_7_Ka_down_color_3);
    color_space_fn(pattern_7_Ka_down_color_4_raw, pattern_7_Ka_down_color_4);
    uv_align_check_pattern(pattern_7_Ka_down_color_0, pattern_7_Ka_down_color_1, pattern_7_Ka_down_color_2, pattern_7_Ka_down_color_3, pattern_7_Ka_down_color_4, pattern_7_Ka_down);


    Color pattern_7_Ka_front_color_0_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_7_Ka_front_color_1_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_7_Ka_front_color_2_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_7_Ka_front_color_3_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_7_Ka_front_color_4_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_7_Ka_front_color_0;
    Color pattern_7_Ka_front_color_1;
    Color pattern_7_Ka_front_color_2;
    Color pattern_7_Ka_front_color_3;
    Color pattern_7_Ka_front_color_4;
    color_space_fn(pattern_7_Ka_front_color_0_raw, pattern_7_Ka_front_color_0);
    color_space_fn(pattern_7_Ka_front_color_1_raw, pattern_7_Ka_front_color_1);
    color_space_fn(pattern_7_Ka_front_color_2_raw, pattern_7_Ka_front_color_2);
    color_space_fn(pattern_7_Ka_front_color_3_raw, pattern_7_Ka_front_color_3);
    color_space_fn(pattern_7_Ka_front_color_4_raw, pattern_7_Ka_front_color_4);
    uv_align_check_pattern(pattern_7_Ka_front_color_0, pattern_7_Ka_front_color_1, pattern_7_Ka_front_color_2, pattern_7_Ka_front_color_3, pattern_7_Ka_front_color_4, pattern_7_Ka_front);


    Color pattern_7_Ka_back_color_0_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_7_Ka_back_color_1_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_7_Ka_back_color_2_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_7_Ka_back_color_3_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_7_Ka_back_color_4_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_7_Ka_back_color_0;
    Color pattern_7_Ka_back_color_1;
    Color pattern_7_Ka_back_color_2;
    Color pattern_7_Ka_back_color_3;
    Color pattern_7_Ka_back_color_4;
    color_space_fn(pattern_7_Ka_back_color_0_raw, pattern_7_Ka_back_color_0);
    color_space_fn(pattern_7_Ka_back_color_1_raw, pattern_7_Ka_back_color_1);
    color_space_fn(pattern_7_Ka_back_color_2_raw, pattern_7_Ka_back_color_2);
    color_space_fn(pattern_7_Ka_back_color_3_raw, pattern_7_Ka_back_color_3);
    color_space_fn(pattern_7_Ka_back_color_4_raw, pattern_7_Ka_back_color_4);
    uv_align_check_pattern(pattern_7_Ka_back_color_0, pattern_7_Ka_back_color_1, pattern_7_Ka_back_color_2, pattern_7_Ka_back_color_3, pattern_7_Ka_back_color_4, pattern_7_Ka_back);



    texture_map_pattern(pattern_7_Ka_right, CUBE_UV_MAP, pattern_7_Ka);
    pattern_set_transform(pattern_7_Ka, transform_pattern_7_Ka);
Matrix transform_pattern_7_Kd;
    matrix_identity(transform_pattern_7_Kd);
    Pattern pattern_7_Kd = array_of_patterns(7);
    Pattern pattern_7_Kd_right = pattern_7_Kd + 1;
    Pattern pattern_7_Kd_left = pattern_7_Kd + 2;
    Pattern pattern_7_Kd_up = pattern_7_Kd + 3;
    Pattern pattern_7_Kd_down = pattern_7_Kd + 4;
    Pattern pattern_7_Kd_front = pattern_7_Kd + 5;
    Pattern pattern_7_Kd_back = pattern_7_Kd + 6;

    Color pattern_7_Kd_right_color_0_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_7_Kd_right_color_1_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_7_Kd_right_color_2_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_7_Kd_right_color_3_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_7_Kd_right_color_4_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_7_Kd_right_color_0;
    Color pattern_7_Kd_right_color_1;
    Color pattern_7_Kd_right_color_2;
    Color pattern_7_Kd_right_color_3;
    Color pattern_7_Kd_right_color_4;
    color_space_fn(pattern_7_Kd_right_color_0_raw, pattern_7_Kd_right_color_0);
    color_space_fn(pattern_7_Kd_right_color_1_raw, pattern_7_Kd_right_color_1);
    color_space_fn(pattern_7_Kd_right_color_2_raw, pattern_7_Kd_right_color_2);
    color_space_fn(pattern_7_Kd_right_color_3_raw, pattern_7_Kd_right_color_3);
    color_space_fn(pattern_7_Kd_right_color_4_raw, pattern_7_Kd_right_color_4);
    uv_align_check_pattern(pattern_7_Kd_right_color_0, pattern_7_Kd_right_color_1, pattern_7_Kd_right_color_2, pattern_7_Kd_right_color_3, pattern_7_Kd_right_color_4, pattern_7_Kd_right);


    Color pattern_7_Kd_left_color_0_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_7_Kd_left_color_1_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_7_Kd_left_color_2_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_7_Kd_left_color_3_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_7_Kd_left_color_4_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_7_Kd_left_color_0;
    Color pattern_7_Kd_left_color_1;
    Color pattern_7_Kd_left_color_2;
    Color pattern_7_Kd_left_color_3;
    Color pattern_7_Kd_left_color_4;
    color_space_fn(pattern_7_Kd_left_color_0_raw, pattern_7_Kd_left_color_0);
    color_space_fn(pattern_7_Kd_left_color_1_raw, pattern_7_Kd_left_color_1);
    color_space_fn(pattern_7_Kd_left_color_2_raw, pattern_7_Kd_left_color_2);
    color_space_fn(pattern_7_Kd_left_color_3_raw, pattern_7_Kd_left_color_3);
    color_space_fn(pattern_7_Kd_left_color_4_raw, pattern_7_Kd_left_color_4);
    uv_align_check_pattern(pattern_7_Kd_left_color_0, pattern_7_Kd_left_color_1, pattern_7_Kd_left_color_2, pattern_7_Kd_left_color_3, pattern_7_Kd_left_color_4, pattern_7_Kd_left);


    Color pattern_7_Kd_up_color_0_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_7_Kd_up_color_1_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_7_Kd_up_color_2_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_7_Kd_up_color_3_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_7_Kd_up_color_4_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_7_Kd_up_color_0;
    Color pattern_7_Kd_up_color_1;
    Color pattern_7_Kd_up_color_2;
    Color pattern_7_Kd_up_color_3;
    Color pattern_7_Kd_up_color_4;
    color_space_fn(pattern_7_Kd_up_color_0_raw, pattern_7_Kd_up_color_0);
    color_space_fn(pattern_7_Kd_up_color_1_raw, pattern_7_Kd_up_color_1);
    color_space_fn(pattern_7_Kd_up_color_2_raw, pattern_7_Kd_up_color_2);
    color_space_fn(pattern_7_Kd_up_color_3_raw, pattern_7_Kd_up_color_3);
    color_space_fn(pattern_7_Kd_up_color_4_raw, pattern_7_Kd_up_color_4);
    uv_align_check_pattern(pattern_7_Kd_up_color_0, pattern_7_Kd_up_color_1, pattern_7_Kd_up_color_2, pattern_7_Kd_up_color_3, pattern_7_Kd_up_color_4, pattern_7_Kd_up);


    Color pattern_7_Kd_down_color_0_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_7_Kd_down_color_1_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_7_Kd_down_color_2_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_7_Kd_down_color_3_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_7_Kd_down_color_4_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_7_Kd_down_color_0;
    Color pattern_7_Kd_down_color_1;
    Color pattern_7_Kd_down_color_2;
    Color pattern_7_Kd_down_color_3;
    Color pattern_7_Kd_down_color_4;
    color_space_fn(pattern_7_Kd_down_color_0_raw, pattern_7_Kd_down_color_0);
    color_space_fn(pattern_7_Kd_down_color_1_raw, pattern_7_Kd_down_color_1);
    color_space_fn(pattern_7_Kd_down_color_2_raw, pattern_7_Kd_down_color_2);
    color_space_fn(pattern_7_Kd_down_color_3_raw, pattern_7_Kd_down_color_3);
    color_space_fn(pattern_7_Kd_down_color_4_raw, pattern_7_Kd_down_color_4);
    uv_align_check_pattern(pattern_7_Kd_down_color_0, pattern_7_Kd_down_color_1, pattern_7_Kd_down_color_2, pattern_7_Kd_down_color_3, pattern_7_Kd_down_color_4, pattern_7_Kd_down);


    Color pattern_7_Kd_front_color_0_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_7_Kd_front_color_1_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color pattern_7_Kd_front_color_2_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_7_Kd_front_color_3_raw = color(1.0000000000, 0.5000000000, 0.0000000000);
    Color pattern_7_Kd_front_color_4_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_7_Kd_front_color_0;
    Color pattern_7_Kd_front_color_1;
    Color pattern_7_Kd_front_color_2;
    Color pattern_7_Kd_front_color_3;
    Color pattern_7_Kd_front_color_4;
    color_space_fn(pattern_7_Kd_front_color_0_raw, pattern_7_Kd_front_color_0);
    color_space_fn(pattern_7_Kd_front_color_1_raw, pattern_7_Kd_front_color_1);
    color_space_fn(pattern_7_Kd_front_color_2_raw, pattern_7_Kd_front_color_2);
    color_space_fn(pattern_7_Kd_front_color_3_raw, pattern_7_Kd_front_color_3);
    color_space_fn(pattern_7_Kd_front_color_4_raw, pattern_7_Kd_front_color_4);
    uv_align_check_pattern(pattern_7_Kd_front_color_0, pattern_7_Kd_front_color_1, pattern_7_Kd_front_color_2, pattern_7_Kd_front_color_3, pattern_7_Kd_front_color_4, pattern_7_Kd_front);


    Color pattern_7_Kd_back_color_0_raw = color(0.0000000000, 1.0000000000, 0.0000000000);
    Color pattern_7_Kd_back_color_1_raw = color(1.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_7_Kd_back_color_2_raw = color(0.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_7_Kd_back_color_3_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color pattern_7_Kd_back_color_4_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color pattern_7_Kd_back_color_0;
    Color pattern_7_Kd_back_color_1;
    Color pattern_7_Kd_back_color_2;
    Color pattern_7_Kd_back_color_3;
    Color pattern_7_Kd_back_color_4;
    color_space_fn(pattern_7_Kd_back_color_0_raw, pattern_7_Kd_back_color_0);
    color_space_fn(pattern_7_Kd_back_color_1_raw, pattern_7_Kd_back_color_1);
    color_space_fn(pattern_7_Kd_back_color_2_raw, pattern_7_Kd_back_color_2);
    color_space_fn(pattern_7_Kd_back_color_3_raw, pattern_7_Kd_back_color_3);
    color_space_fn(pattern_7_Kd_back_color_4_raw, pattern_7_Kd_back_color_4);
    uv_align_check_pattern(pattern_7_Kd_back_color_0, pattern_7_Kd_back_color_1, pattern_7_Kd_back_color_2, pattern_7_Kd_back_color_3, pattern_7_Kd_back_color_4, pattern_7_Kd_back);



    texture_map_pattern(pattern_7_Kd_right, CUBE_UV_MAP, pattern_7_Kd);
    pattern_set_transform(pattern_7_Kd, transform_pattern_7_Kd);
    Pattern pattern_7_Ks = NULL;
    Pattern pattern_7_Ns = NULL;
    Pattern pattern_7_bump = NULL;
    Pattern pattern_7_disp = NULL;
    Pattern pattern_7_refl = NULL;
    Pattern pattern_7_d = NULL;
    Color material_7_color_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color material_7_reflective = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_7_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_7 = material_alloc();
    color_space_fn(material_7_color_raw, material_7->Ka);
    color_space_fn(material_7_color_raw, material_7->Kd);
    color_space_fn(material_7_color_raw, material_7->Ks);
    color_scale(material_7->Ka, 0.2000000000);
    color_scale(material_7->Kd, 0.8000000000);
    color_scale(material_7->Ks, 0.0000000000);
    rgb_to_rgb(material_7_reflective, material_7->refl);
    rgb_to_rgb(material_7_refractive, material_7->Tf);
    material_7->reflective = material_7_reflective[0] > 0.0
                             || material_7_reflective[1] > 0.0
                             || material_7_reflective[2] > 0.0;

    material_7->Tr = 0.0000000000;
    material_7->Ns = 200.0000000000;
    material_7->Ni = 1.0000000000;
    material_7->casts_shadow = true;
    material_set_pattern(material_7, map_Ka, pattern_7_Ka);
    material_set_pattern(material_7, map_Kd, pattern_7_Kd);
    material_set_pattern(material_7, map_Ks, pattern_7_Ks);
    material_set_pattern(material_7, map_Ns, pattern_7_Ns);
    material_set_pattern(material_7, map_d, pattern_7_d);
    material_set_pattern(material_7, map_bump, pattern_7_bump);
    material_set_pattern(material_7, map_disp, pattern_7_disp);
    material_set_pattern(material_7, map_refl, pattern_7_refl);

    Matrix transform_7, transform_7_tmp;
    matrix_identity(transform_7);
    matrix_rotate_y(5.4978000000, transform_7_tmp);
    transform_chain(transform_7_tmp, transform_7);
    matrix_rotate_x(-0.7854000000, transform_7_tmp);
    transform_chain(transform_7_tmp, transform_7);
    matrix_translate(6.0000000000, -2.0000000000, 0.0000000000, transform_7_tmp);
    transform_chain(transform_7_tmp, transform_7);

    Shape shape_7 = all_shapes + 7;
    cube(shape_7);
    shape_set_material(shape_7, material_7);
    shape_set_transform(shape_7, transform_7);

    /* end shape 7 */
    /* end shapes */

    Shape world_group = array_of_shapes(1);
    group(world_group, all_shapes, 8);
    printf("Balancing scene...");
    fflush(stdout);
    world_group->divide(world_group, global_config.scene.divide_threshold);
    printf("Done!\n");
    fflush(stdout);

    World w = world();
    w->lights = all_lights;
    w->lights_num = 4;
    w->shapes = world_group;
    w->shapes_num = 1;
    w->global_config = &global_config;

    if (global_config.illumination.gi.photon_count > 0 && (global_config.illumination.include_global  || global_config.illumination.debug_visualize_photon_map || global_config.illumination.debug_visualize_soft_indirect)) {
        w->photon_maps = array_of_photon_maps(3);
        printf("Tracing photons...");
        fflush(stdout);
        int i;
        for (i = 0; i < 3; ++i) {
            init_Photon_map(global_config.illumination.gi.photon_count, w->photon_maps + i);
        }
        trace_photons(w, 3, global_config.illumination.gi.include_caustics, global_config.illumination.gi.include_final_gather);
        printf("Done!\n");
        fflush(stdout);
    } else {
        w->photon_maps = NULL;
        printf("Skipping photon tracing because photon_count is 0.\n");
        fflush(stdout);
    }

    Canvas c = render_multi(cam, w, cam->usteps, cam->vsteps, cam->aperture.jitter);

    write_ppm_file(c, true, global_config.output.file_path);
    write_png(c, global_config.output.file_path);

    canvas_free(c);

    return 0;
}

